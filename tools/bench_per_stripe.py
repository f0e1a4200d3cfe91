#!/usr/bin/env python3
"""Per-stripe ErasureScheme calls through the C-ABI: what an unchanged Go
caller costs before the batch interfaces are wired in.

segmentupload's EncodedReader calls EncodeSingle once per (piece, stripe)
(private/storage/streams/segmentupload/encode.go:58) from up to 300 piece
goroutines (private/testuplink/uplink.go:83); StripeReader calls Rebuild once
per stripe (private/eestream/stripe.go:407-413).  This measures, for
RS(29,80) and 7424-byte stripes:
  * ec_encode_single / ec_rebuild latency from one thread and aggregate
    calls/s from T threads (ctypes releases the GIL, so the calls overlap in
    the library);
  * the same calls on the CPU oracle (the reference-shaped per-call work) for
    the crossover.
Writes one JSON line.  Run on a GPU box: python tools/bench_per_stripe.py
"""
from __future__ import annotations

import ctypes
import json
import os
import sys
import threading
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

from uplink_amd import _native  # noqa: E402

K, N, ESS = 29, 80, 256
STRIPE = K * ESS


def run_threads(nthreads: int, seconds: float, make_call):
    """Aggregate calls/s of `nthreads` threads each looping its own call."""
    stop = time.perf_counter() + seconds
    counts = [0] * nthreads
    lat = [0.0] * nthreads

    def worker(t):
        call = make_call(t)
        n = 0
        t0 = time.perf_counter()
        while time.perf_counter() < stop:
            call(n)
            n += 1
        counts[t] = n
        lat[t] = (time.perf_counter() - t0) / max(n, 1)

    th = [threading.Thread(target=worker, args=(t,)) for t in range(nthreads)]
    t0 = time.perf_counter()
    for x in th:
        x.start()
    for x in th:
        x.join()
    wall = time.perf_counter() - t0
    return {"threads": nthreads, "calls_per_s": round(sum(counts) / wall, 1),
            "mean_latency_us": round(sum(lat) / nthreads * 1e6, 2),
            "MB_per_s_of_stripes": round(sum(counts) * STRIPE / wall / 1e6, 1)}


def main():
    L = _native.load()
    ctx = ctypes.c_void_p()
    assert L.ec_create(K, N, ESS, ctypes.byref(ctx)) == 0
    rng = np.random.default_rng(1)
    stripes = [rng.integers(0, 256, STRIPE, dtype=np.uint8) for _ in range(64)]
    outs = [np.empty(ESS, dtype=np.uint8) for _ in range(512)]
    # shares of every stripe (for the rebuild calls): all 80
    allsh = []
    for s in stripes:
        o = np.empty(N * ESS, dtype=np.uint8)
        assert L.ec_encode(ctx, s.ctypes.data, STRIPE, o.ctypes.data) == 0
        allsh.append(o.reshape(N, ESS))
    parity = list(range(N - K, N))

    def gpu_encode(t):
        out = outs[t % len(outs)]

        def call(i):
            s = stripes[(t + i) % len(stripes)]
            assert L.ec_encode_single(ctx, s.ctypes.data, STRIPE, out.ctypes.data, ESS, K + (i % (N - K))) == 0
        return call

    def gpu_rebuild(t):
        dst = np.empty(STRIPE, dtype=np.uint8)

        def call(i):
            sh = allsh[(t + i) % len(allsh)]
            nums = (ctypes.c_int * K)(*parity)
            ptrs = (ctypes.c_void_p * K)(*[sh[j].ctypes.data for j in parity])
            assert L.ec_rebuild(ctx, K, nums, ptrs, ESS, dst.ctypes.data) == 0
        return call

    from oracle import oracle as O
    f = O.FEC(K, N)

    def cpu_encode(t):
        def call(i):
            f.encode_single(stripes[(t + i) % len(stripes)], K + (i % (N - K)))
        return call

    def cpu_rebuild(t):
        def call(i):
            sh = allsh[(t + i) % len(allsh)]
            f.rebuild(parity, [sh[j] for j in parity])
        return call

    res = {"config": "RS(29,80), ess 256, one 7424-byte stripe per call", "encode_single": [], "rebuild": [],
           "cpu_oracle_encode_single": [], "cpu_oracle_rebuild": []}
    for T in (1, 4, 16, 64):
        res["encode_single"].append(run_threads(T, 2.0, gpu_encode))
        res["rebuild"].append(run_threads(T, 2.0, gpu_rebuild))
    for T in (1, 16):
        res["cpu_oracle_encode_single"].append(run_threads(T, 1.0, cpu_encode))
        res["cpu_oracle_rebuild"].append(run_threads(T, 1.0, cpu_rebuild))
    L.ec_destroy(ctx)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
