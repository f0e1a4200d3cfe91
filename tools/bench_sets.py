#!/usr/bin/env python3
"""Fresh share sets, the way uplink decodes: every
segment of a download comes with whichever 29 pieces answered first
(private/eestream/stripe.go:314-354), so its decode plan is new.

  * batch: ec_rebuild_segments_sets, 32 RS(29,80) 64 MiB segments per call,
    32 fresh seeded 29-subsets per call; HIP-event time per call on the
    stream (launches back to back) and wall time per call.
  * single: one segment, a fresh set, wall clock per call (launch + sync), the
    time until the call returns, and a one-element torch kernel's wall clock
    (this box's floor for a launch and a synchronisation).
  * batched API (ec_rebuild_segments_batched) on a fresh set: first, second
    and warm launch of the set, wall clock, one segment and 16.
Run on the GPU box: python tools/bench_sets.py [--reps N]"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from uplink_amd import _native  # noqa: E402

K, N, ESS = 29, 80, 256
NSTRIPES = (64 * 2**20 + 4 + K * ESS - 1) // (K * ESS)
SPAD, PLEN = NSTRIPES * K * ESS, NSTRIPES * ESS
PEAK = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=24)
    ap.add_argument("--nseg", type=int, default=32)
    args = ap.parse_args()
    torch.cuda.set_device(0)
    L = _native.load()
    ctx = ctypes.c_void_p()
    assert L.ec_create(K, N, ESS, ctypes.byref(ctx)) == 0
    dev = torch.device("cuda", 0)
    nseg = args.nseg
    segs = torch.randint(0, 256, (nseg, SPAD), dtype=torch.uint8, device=dev)
    pcs = torch.empty((nseg, N, PLEN), dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream()
    sptr = st.cuda_stream
    assert L.ec_encode_segments(ctx, segs.data_ptr(), nseg, NSTRIPES, pcs.data_ptr(), 0, sptr) == 0
    outs = torch.empty_like(segs)
    rng = np.random.default_rng(2905)

    def fresh(count):
        return [sorted(int(x) for x in rng.permutation(N)[:K]) for _ in range(count)]

    def sets_args(sets, out=outs):
        """the call's ctypes arrays, made ahead of the timed calls (a Go caller has its slices)"""
        n = len(sets)
        nsh = (ctypes.c_int * n)(*[K] * n)
        flat = [x for s in sets for x in s]
        nums = (ctypes.c_int * len(flat))(*flat)
        ptrs = (ctypes.c_void_p * len(flat))(*[pcs[g].data_ptr() + x * PLEN for g, s in enumerate(sets) for x in s])
        optr = (ctypes.c_void_p * n)(*[out[g].data_ptr() for g in range(n)])
        return n, nsh, nums, ptrs, optr

    def sets_go(a):
        n, nsh, nums, ptrs, optr = a
        rc = L.ec_rebuild_segments_sets(ctx, n, nsh, nums, ptrs, NSTRIPES, optr, sptr)
        assert rc == 0, _native.strerror(rc)

    def sets_call(sets, out=outs):
        sets_go(sets_args(sets, out))

    res = {}
    # warm-up (kernels loaded, slots allocated)
    for _ in range(3):
        sets_call(fresh(nseg))
    torch.cuda.synchronize()
    outs.zero_()
    sets_call(fresh(nseg))
    torch.cuda.synchronize()
    ok = bool(torch.equal(outs, segs))
    # batch: back to back, events around each call
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.reps + 1)]
    all_sets = [fresh(nseg) for _ in range(args.reps)]
    all_args = [sets_args(x) for x in all_sets]
    # clock settle at the timed loop's duty cycle (arrays made beforehand, calls back to back)
    t_end = time.perf_counter() + 0.3
    i = 0
    while time.perf_counter() < t_end:
        sets_go(all_args[i % args.reps])
        i += 1
    torch.cuda.synchronize()
    ev[0].record(st)
    t0 = time.perf_counter()
    for i in range(args.reps):
        sets_go(all_args[i])
        ev[i + 1].record(st)
    ev[-1].synchronize()
    wall = (time.perf_counter() - t0) / args.reps
    per = [ev[i].elapsed_time(ev[i + 1]) * 1e-3 for i in range(args.reps)]
    t = float(np.median(per))
    alg = nseg * 2 * SPAD
    res["batch"] = {"segments_per_call": nseg, "us_per_call_median": round(t * 1e6, 1),
                    "us_per_call_mean": round(float(np.mean(per)) * 1e6, 1),
                    "us_per_segment": round(t / nseg * 1e6, 2), "GBps": round(alg / t / 1e9, 1),
                    "frac": round(alg / t / 1e9 / PEAK, 4), "wall_us_per_call": round(wall * 1e6, 1),
                    "m_of_sets": sorted(int(sum(1 for x in s if x >= K)) for s in all_sets[0])}
    # host time of one 32-segment call (the launch call alone, the ring empty)
    host = []
    for a in [sets_args(fresh(nseg)) for _ in range(6)]:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sets_go(a)
        host.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
    res["batch"]["host_us_per_call_median"] = round(float(np.median(host)) * 1e6, 1)
    # Decode with error detection over the same segments, each from a fresh set of k+4 clean shares
    # (ec_decode_segments_sets: returns when done, so wall clock per call)
    def dec_args(sets):
        n = len(sets)
        flat = [x for st_ in sets for x in st_]
        return (n, (ctypes.c_int * n)(*[len(st_) for st_ in sets]), (ctypes.c_int * len(flat))(*flat),
                (ctypes.c_void_p * len(flat))(*[pcs[g].data_ptr() + x * PLEN for g, st_ in enumerate(sets) for x in st_]),
                (ctypes.c_void_p * n)(*[outs[g].data_ptr() for g in range(n)]))
    dsets = [[[int(x) for x in rng.permutation(N)[:K + 4]] for _ in range(nseg)] for _ in range(args.reps)]
    dargs = [dec_args(x) for x in dsets]
    for a in dargs[:3]:
        assert L.ec_decode_segments_sets(ctx, *a[:4], NSTRIPES, a[4], sptr) == 0
    dw = []
    dec_ok = True
    for a in dargs:
        outs.zero_()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        assert L.ec_decode_segments_sets(ctx, *a[:4], NSTRIPES, a[4], sptr) == 0
        dw.append(time.perf_counter() - t0)
        dec_ok = dec_ok and bool(torch.equal(outs[:nseg], segs[:nseg]))  # (after the timed call)
    td = float(np.median(dw))
    dalg = nseg * (PLEN * (K + 4) + SPAD)
    res["decode_sets_k+4"] = {"segments_per_call": nseg, "wall_us_per_call_median": round(td * 1e6, 1),
                              "us_per_segment": round(td / nseg * 1e6, 2), "frac": round(dalg / td / 1e9 / PEAK, 4),
                              "verified": dec_ok,
                              "note": "fresh seeded (k+4)-subsets, clean; bytes = the k+4 pieces read + the segment"}
    # the same 32 segments from ONE share set, warm plan, back to back on the stream: the
    # straight-line body and the jump-table body of ec_rebuild_segments_batched, timed as above
    one = all_sets[0][0]
    cn = (ctypes.c_int * K)(*one)
    cp = (ctypes.c_void_p * K)(*[pcs[0].data_ptr() + x * PLEN for x in one])
    assert L.ec_prepare_rebuild(ctx, K, cn, 1) == 1
    for body, name in ((_native.EC_BODY_AUTO, "straight_line"), (_native.EC_BODY_JUMP_TABLE, "jump_table")):
        assert L.ec_set_body(ctx, body) == 0

        def one_set():
            assert L.ec_rebuild_segments_batched(ctx, K, cn, cp, NSTRIPES, nseg, N * PLEN, SPAD, outs.data_ptr(),
                                                 sptr) == 0
        for _ in range(3):
            one_set()
        torch.cuda.synchronize()
        t_end = time.perf_counter() + 0.3
        while time.perf_counter() < t_end:
            one_set()
        torch.cuda.synchronize()
        ev[0].record(st)
        for i in range(args.reps):
            one_set()
            ev[i + 1].record(st)
        ev[-1].synchronize()
        per1 = [ev[i].elapsed_time(ev[i + 1]) * 1e-3 for i in range(args.reps)]
        t1 = float(np.median(per1))
        res[f"one_set_{name}"] = {"m": int(sum(1 for x in one if x >= K)), "us_per_call_median": round(t1 * 1e6, 1),
                                  "frac": round(alg / t1 / 1e9 / PEAK, 4), "body": int(L.ec_last_body(ctx))}
    assert L.ec_set_body(ctx, _native.EC_BODY_AUTO) == 0
    torch.cuda.synchronize()
    # single segment, fresh set, synchronous wall clock
    walls, calls, floor = [], [], []
    tiny = torch.zeros(1, dtype=torch.int32, device=outs.device)
    for i in range(args.reps * 4):
        a1 = sets_args(fresh(1), outs)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sets_go(a1)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        walls.append(time.perf_counter() - t0)
        calls.append(t1 - t0)
        # this box's floor for one launch and a synchronisation, as Python sees it
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tiny.add_(1)
        torch.cuda.synchronize()
        floor.append(time.perf_counter() - t0)
    ev2 = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    s1s = [sets_args(fresh(1), outs) for _ in range(args.reps)]
    torch.cuda.synchronize()
    ev2[0].record(st)
    for a1 in s1s:
        sets_go(a1)
    ev2[1].record(st)
    ev2[1].synchronize()
    b2b = ev2[0].elapsed_time(ev2[1]) * 1e-3 / args.reps
    res["single"] = {"wall_us_median": round(float(np.median(walls)) * 1e6, 1),
                     "wall_us_min": round(min(walls) * 1e6, 1),
                     "call_returns_us_median": round(float(np.median(calls)) * 1e6, 1),
                     "tiny_kernel_wall_us_median": round(float(np.median(floor)) * 1e6, 1),
                     "stream_us_back_to_back": round(b2b * 1e6, 1),
                     "frac_back_to_back": round(2 * SPAD / b2b / 1e9 / PEAK, 4)}
    # the batched single-set API on fresh sets: first / second / warm, wall clock
    for n in (1, 16):
        rows = []
        for i in range(args.reps):
            nums = fresh(1)[0]
            cn = (ctypes.c_int * K)(*nums)
            cp = (ctypes.c_void_p * K)(*[pcs[0].data_ptr() + x * PLEN for x in nums])
            t = []
            for rep in range(3):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                assert L.ec_rebuild_segments_batched(ctx, K, cn, cp, NSTRIPES, n, N * PLEN, SPAD, outs.data_ptr(),
                                                     sptr) == 0
                torch.cuda.synchronize()
                t.append(time.perf_counter() - t0)
                if rep == 1:
                    L.ec_prepare_rebuild(ctx, K, cn, 1)
            rows.append(t)
        a = np.array(rows) * 1e6
        res[f"batched_api_{n}seg"] = {"first_us": round(float(np.median(a[:, 0])), 1),
                                      "second_us": round(float(np.median(a[:, 1])), 1),
                                      "warm_us": round(float(np.median(a[:, 2])), 1),
                                      "second_max_us": round(float(a[:, 1].max()), 1)}
    res["verified"] = ok
    print(json.dumps(res))
    L.ec_destroy(ctx)


if __name__ == "__main__":
    main()
