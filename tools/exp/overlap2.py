#!/usr/bin/env python3
"""Experiment (GPU box): encode of batch i+1 on one stream while batch i is
rebuilt on another, with the current kernels (one-workgroup-per-tile
rebuild, persistent encoder), against the bench's single-stream order.
RS(29,80), 16 x 64 MiB segments per launch, pool of 2 slots, the bench's 8
share sets.  Prints wall time per launch pair for both orders, alternated.
python tools/exp/overlap2.py [pairs]"""
import ctypes
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from uplink_amd import _native  # noqa: E402

K, N, ESS, B = 29, 80, 256, 16
NSTRIPES = 9040
S_PAD, PIECE = NSTRIPES * K * ESS, NSTRIPES * ESS


def main(pairs):
    L = _native.load()
    ctx = ctypes.c_void_p()
    assert L.ec_create(K, N, ESS, ctypes.byref(ctx)) == 0
    dev = torch.device("cuda", 0)
    segs = [torch.randint(0, 256, (B, S_PAD), dtype=torch.uint8, device=dev) for _ in range(2)]
    pieces = [torch.empty((B, N, PIECE), dtype=torch.uint8, device=dev) for _ in range(2)]
    outs = [torch.empty((B, S_PAD), dtype=torch.uint8, device=dev) for _ in range(2)]
    rng = np.random.default_rng(29)
    sets = [list(range(N - K, N))] + [sorted(rng.choice(N, K, replace=False).tolist()) for _ in range(7)]
    nums_c = [(ctypes.c_int * K)(*s) for s in sets]
    ptrs_c = [[(ctypes.c_void_p * K)(*[p.data_ptr() + j * PIECE for j in s]) for s in sets] for p in pieces]
    sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)

    def enc(slot, st):
        assert L.ec_encode_segments(ctx, segs[slot].data_ptr(), B, NSTRIPES, pieces[slot].data_ptr(), 0,
                                    st.cuda_stream) == 0

    def dec(slot, i, st):
        assert L.ec_rebuild_segments_batched(ctx, K, nums_c[i], ptrs_c[slot][i], NSTRIPES, B, N * PIECE, S_PAD,
                                             outs[slot].data_ptr(), st.cuda_stream) == 0

    def sequential(n):
        for p in range(n):
            enc(p % 2, sa)
            dec(p % 2, p % 8, sa)

    def overlapped(n):
        # encode(p) on sa after decode(p-2) (same slot); decode(p) on sb after encode(p)
        done_dec = [None, None]
        for p in range(n):
            slot = p % 2
            if done_dec[slot] is not None:
                sa.wait_event(done_dec[slot])
            enc(slot, sa)
            e = torch.cuda.Event()
            e.record(sa)
            sb.wait_event(e)
            dec(slot, p % 8, sb)
            d = torch.cuda.Event()
            d.record(sb)
            done_dec[slot] = d

    for f in (sequential, overlapped):  # warm-up and plans
        f(16)
    torch.cuda.synchronize()
    for rep in range(3):
        for name, f in (("sequential", sequential), ("overlapped", overlapped)):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            f(pairs)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            print(json.dumps({"order": name, "rep": rep, "us_per_pair": round(dt / pairs * 1e6, 1),
                              "GiB_per_s": round(pairs * B * S_PAD / 2**30 / dt, 1)}), flush=True)
    for s in range(2):
        enc(s, sa)
        dec(s, 0, sa)
    torch.cuda.synchronize()
    print(json.dumps({"verified": all(bool(torch.equal(outs[s], segs[s])) for s in range(2))}))
    L.ec_destroy(ctx)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 64)
