#!/usr/bin/env python3
"""Why the share-set decode is slower inside the bench's encode/decode
alternation than back to back: HIP-event time of one 32-segment
ec_rebuild_segments_sets call (fresh sets) and of the warm straight-line
rebuild of one set, each (a) back to back, (b) right after a full RS(29,80)
encode launch, (c) right after a device copy of similar length, (d) after the
GPU idled ~1.5 ms, (e) right after a one-segment encode (every CU runs the
encoder's code, 1/32 of its heat), (f) after a full encode and then a
one-segment share-set decode (the leaves back in the instruction caches, the
heat unchanged).  Prints one JSON line."""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from uplink_amd import _native  # noqa: E402

K, N, ESS, NSTRIPES = 29, 80, 256, 9040
SPAD, PLEN, B = NSTRIPES * K * ESS, NSTRIPES * ESS, 32


def main():
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    L = _native.load()
    ctx = ctypes.c_void_p()
    assert L.ec_create(K, N, ESS, ctypes.byref(ctx)) == 0
    st = torch.cuda.current_stream()
    sp = st.cuda_stream
    segs = torch.randint(0, 256, (B, SPAD), dtype=torch.uint8, device=dev)
    pcs = torch.empty((B, N, PLEN), dtype=torch.uint8, device=dev)
    outs = torch.empty_like(segs)
    cp_src = torch.empty(4 << 30, dtype=torch.uint8, device=dev)
    cp_dst = torch.empty_like(cp_src)
    rng = np.random.default_rng(77)

    def enc():
        assert L.ec_encode_segments(ctx, segs.data_ptr(), B, NSTRIPES, pcs.data_ptr(), 0, sp) == 0

    def enc1():
        assert L.ec_encode_segments(ctx, segs.data_ptr(), 1, NSTRIPES, pcs.data_ptr(), 0, sp) == 0

    def sets_args():
        sets = [sorted(int(x) for x in rng.permutation(N)[:K]) for _ in range(B)]
        flat = [x for s in sets for x in s]
        return ((ctypes.c_int * B)(*[K] * B), (ctypes.c_int * len(flat))(*flat),
                (ctypes.c_void_p * len(flat))(*[pcs[g].data_ptr() + x * PLEN for g, s in enumerate(sets) for x in s]),
                (ctypes.c_void_p * B)(*[outs[g].data_ptr() for g in range(B)]))
    pool = [sets_args() for _ in range(24)]

    def dec_sets(i):
        a = pool[i % len(pool)]
        assert L.ec_rebuild_segments_sets(ctx, B, a[0], a[1], a[2], NSTRIPES, a[3], sp) == 0
    s1 = sorted(int(x) for x in rng.permutation(N)[:K])
    a1 = ((ctypes.c_int * 1)(K), (ctypes.c_int * K)(*s1), (ctypes.c_void_p * K)(*[pcs[1].data_ptr() + x * PLEN for x in s1]),
          (ctypes.c_void_p * 1)(outs[1].data_ptr()))

    def dec_sets1():
        assert L.ec_rebuild_segments_sets(ctx, 1, a1[0], a1[1], a1[2], NSTRIPES, a1[3], sp) == 0
    one = sorted(int(x) for x in rng.permutation(N)[:K])
    cn = (ctypes.c_int * K)(*one)
    cptr = (ctypes.c_void_p * K)(*[pcs[0].data_ptr() + x * PLEN for x in one])

    def dec_sl(i):
        assert L.ec_rebuild_segments_batched(ctx, K, cn, cptr, NSTRIPES, B, N * PLEN, SPAD, outs.data_ptr(), sp) == 0

    def copy():
        cp_dst.copy_(cp_src)

    def pre(mode):
        if mode in ("after_encode", "after_encode_and_one_segment"):
            enc()
        elif mode == "after_copy":
            copy()
        elif mode == "after_small_encode":
            enc1()
        if mode == "after_encode_and_one_segment":
            dec_sets1()

    enc()
    dec_sl(0)
    L.ec_prepare_rebuild(ctx, K, cn, 1)
    res = {}
    for name, dec in (("sets", dec_sets), ("straight_line", dec_sl)):
        for mode in ("back_to_back", "after_encode", "after_copy", "after_idle", "after_small_encode",
                     "after_encode_and_one_segment"):
            t_end = time.perf_counter() + 0.4
            i = 0
            while time.perf_counter() < t_end:  # settle in the same duty cycle
                pre(mode)
                dec(i)
                i += 1
                if mode == "after_idle":
                    torch.cuda.synchronize()
                    time.sleep(0.0015)
            torch.cuda.synchronize()
            per = []
            for r in range(16):
                pre(mode)
                if mode == "after_idle":
                    torch.cuda.synchronize()
                    time.sleep(0.0015)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                dec(r)
                e1.record(st)
                per.append((e0, e1))
            torch.cuda.synchronize()
            t = sorted(a.elapsed_time(b) * 1e3 for a, b in per)
            res[f"{name}/{mode}"] = round(t[len(t) // 2], 1)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record(st)
    copy()
    ev[1].record(st)
    torch.cuda.synchronize()
    res["copy_us"] = round(ev[0].elapsed_time(ev[1]) * 1e3, 1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
