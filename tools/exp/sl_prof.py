#!/usr/bin/env python3
"""Profiling driver (GPU box, under rocprofv3): RS(29,80) rebuilds of 16 x 64 MiB
segments, 20 launches per (share set, body), the straight-line and the
jump-table bodies one after the other, so per-kernel counters separate by
kernel name (rs_matmul_jt<NW, true> / <NW, false>).
python tools/exp/sl_prof.py [set ...]   (bench share-set indices, default 0 1)"""
import ctypes
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, HERE)

import torch  # noqa: E402

from sl_bench import sets_of  # noqa: E402
from uplink_amd import _native  # noqa: E402


def main(which):
    L = _native.load()
    s = torch.cuda.current_stream().cuda_stream
    k, n, ess, nseg = 29, 80, 256, 16
    stripes = 9040
    spad, plen = stripes * k * ess, stripes * ess
    ctx = ctypes.c_void_p()
    assert L.ec_create(k, n, ess, ctypes.byref(ctx)) == 0
    segs = torch.randint(0, 256, (nseg, spad), dtype=torch.uint8, device="cuda")
    pcs = torch.empty((nseg, n, plen), dtype=torch.uint8, device="cuda")
    assert L.ec_encode_segments(ctx, segs.data_ptr(), nseg, stripes, pcs.data_ptr(), 0, s) == 0
    back = torch.empty((nseg, spad), dtype=torch.uint8, device="cuda")
    sets = sets_of(k, n)
    for body in (_native.EC_BODY_STRAIGHT_LINE, _native.EC_BODY_JUMP_TABLE):
        assert L.ec_set_body(ctx, body) == 0
        for si in which:
            nums = sets[si]
            nc = (ctypes.c_int * k)(*nums)
            pp = (ctypes.c_void_p * k)(*[pcs.data_ptr() + j * plen for j in nums])
            for _ in range(20):
                assert L.ec_rebuild_segments_batched(ctx, k, nc, pp, stripes, nseg, n * plen, spad, back.data_ptr(),
                                                     s) == 0
            torch.cuda.synchronize()
            assert torch.equal(back, segs)
    L.ec_destroy(ctx)
    print("ok")


if __name__ == "__main__":
    main([int(x) for x in sys.argv[1:]] or [0, 1])
