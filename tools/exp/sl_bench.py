#!/usr/bin/env python3
"""Straight-line rebuild bodies against the jump table (GPU box).

1. One small rebuild (RS(29,80), 64 stripes, all-parity share set) with
   EC_BODY_STRAIGHT_LINE, checked against the input: the first run of
   generated code.
2. The bench's shape: 16 x 64 MiB RS(29,80) segments rebuilt from each of the
   bench's 8 share sets with both bodies (HIP events, 10 launches each), the
   outputs compared with the segments; the time the first straight-line launch
   of a plan takes (code generation + module load + launch).
3. The reference benchmark configurations' all-parity rebuilds.
python tools/exp/sl_bench.py [--small-only | --k29-only | --big]
"""
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

ESS = 256


def sets_of(k, n):
    rng = np.random.default_rng(29)
    sets = [list(range(n - k, n))]
    for _ in range(7):
        sets.append(sorted(rng.choice(n, k, replace=False).tolist()))
    return sets


def run(L, k, n, nseg, raw, s, small=False):
    dev = torch.device("cuda", 0)
    stripe = k * ESS
    stripes = (raw + 4 + stripe - 1) // stripe
    spad, plen = stripes * stripe, stripes * ESS
    ctx = ctypes.c_void_p()
    assert L.ec_create(k, n, ESS, ctypes.byref(ctx)) == 0
    segs = torch.randint(0, 256, (nseg, spad), dtype=torch.uint8, device=dev)
    pcs = torch.empty((nseg, n, plen), dtype=torch.uint8, device=dev)
    assert L.ec_encode_segments(ctx, segs.data_ptr(), nseg, stripes, pcs.data_ptr(), 0, s) == 0
    back = torch.empty((nseg, spad), dtype=torch.uint8, device=dev)
    out = []
    for si, nums in enumerate(sets_of(k, n)[: 1 if small else 8]):
        nc = (ctypes.c_int * k)(*nums)
        pp = (ctypes.c_void_p * k)(*[pcs.data_ptr() + j * plen for j in nums])
        m = k - sum(1 for x in nums if x < k)

        def dec():
            rc = L.ec_rebuild_segments_batched(ctx, k, nc, pp, stripes, nseg, n * plen, spad, back.data_ptr(), s)
            assert rc == 0, rc

        res = {"k": k, "n": n, "set": si, "m": m}
        for body, name in ((_native.EC_BODY_JUMP_TABLE, "jt"), (_native.EC_BODY_STRAIGHT_LINE, "sl")):
            assert L.ec_set_body(ctx, body) == 0
            back.zero_()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            dec()
            torch.cuda.synchronize()
            first = time.perf_counter() - t0
            ok = bool(torch.equal(back, segs))
            used = L.ec_last_body(ctx)
            if small:
                res.update({f"{name}_ok": ok, f"{name}_used": used, f"{name}_first_ms": round(first * 1e3, 2)})
                continue
            for _ in range(3):
                dec()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                dec()
            e1.record()
            e1.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / 10 / nseg
            ok = ok and bool(torch.equal(back, segs))
            res.update({f"{name}_us_per_segment": round(us, 2), f"{name}_TBps": round(2 * spad / us / 1e6, 3),
                        f"{name}_ok": ok, f"{name}_used": used, f"{name}_first_ms": round(first * 1e3, 2)})
        print(json.dumps(res), flush=True)
        out.append(res)
    L.ec_destroy(ctx)
    return out


def main():
    L = _native.load()
    s = torch.cuda.current_stream().cuda_stream
    run(L, 29, 80, 1, 64 * 29 * ESS - 4, s, small=True)
    if "--small-only" in sys.argv:
        return
    if "--big" in sys.argv:  # plans of the 2-MiB code region
        for k, n in ((64, 96), (128, 256)):
            run(L, k, n, 4, 64 << 20, s)
        return
    run(L, 29, 80, 16, 64 << 20, s)
    if "--k29-only" in sys.argv:
        return
    for k, n in ((20, 50), (30, 60), (50, 80)):
        r = run(L, k, n, 8, 64 << 20, s)
        del r


if __name__ == "__main__":
    main()
