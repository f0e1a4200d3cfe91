#!/usr/bin/env python3
"""Probe (GPU box): how fast does a compile-time-coefficient body run a
29-input x m-output product, next to the runtime-matrix rebuild of the same
shape?  The parity-only encode of RS(29, 29+m) (hiprtc-compiled) has exactly
the rebuild's shape for m missing data shares (29 reads, m writes per column),
with the coefficients baked into the code instead of called through the jump
table.  Prints one JSON line per m:  python tools/exp/sl_probe.py [m ...]
"""
import ctypes
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from uplink_amd import _native  # noqa: E402

K, ESS, NSEG = 29, 256, 16


def timed(fn, it=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / it / NSEG


def main(ms):
    L = _native.load()
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream().cuda_stream
    stripes = (64 << 20) // (K * ESS) + 1
    spad, plen = stripes * K * ESS, stripes * ESS
    segs = torch.randint(0, 256, (NSEG, spad), dtype=torch.uint8, device=dev)
    for m in ms:
        n = K + m
        ctx = ctypes.c_void_p()
        assert L.ec_create(K, n, ESS, ctypes.byref(ctx)) == 0
        L.ec_prepare_encoder(ctx, 1)
        par = torch.empty((NSEG, m, plen), dtype=torch.uint8, device=dev)
        t_po = timed(lambda: L.ec_encode_segments(ctx, segs.data_ptr(), NSEG, stripes, par.data_ptr(),
                                                   _native.EC_FLAG_PARITY_ONLY, s))
        # the rebuild of the same shape: RS(29,80) from m parity pieces + 29-m data pieces
        pcs = torch.empty((NSEG, 80, plen), dtype=torch.uint8, device=dev)
        c80 = ctypes.c_void_p()
        assert L.ec_create(K, 80, ESS, ctypes.byref(c80)) == 0
        assert L.ec_encode_segments(c80, segs.data_ptr(), NSEG, stripes, pcs.data_ptr(), 0, s) == 0
        nums = list(range(m, K)) + list(range(80 - m, 80))
        nc = (ctypes.c_int * K)(*nums)
        pp = (ctypes.c_void_p * K)(*[pcs.data_ptr() + j * plen for j in nums])
        back = torch.empty((NSEG, spad), dtype=torch.uint8, device=dev)
        t_rb = timed(lambda: L.ec_rebuild_segments_batched(c80, K, nc, pp, stripes, NSEG, 80 * plen, spad,
                                                           back.data_ptr(), s))
        ok = bool(torch.equal(back, segs))
        print(json.dumps({"m": m, "kernel": L.ec_encode_kernel_name(ctx).decode(),
                          "compile_time_body_us_per_segment": round(t_po, 2),
                          "compile_time_TBps": round(2 * spad / t_po / 1e6, 3) if m == K else None,
                          "jt_rebuild_us_per_segment": round(t_rb, 2), "rebuild_ok": ok}), flush=True)
        del par, pcs, back
        L.ec_destroy(ctx)
        L.ec_destroy(c80)


if __name__ == "__main__":
    main([int(x) for x in sys.argv[1:]] or [29, 22, 16, 8])
