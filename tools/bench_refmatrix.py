#!/usr/bin/env python3
"""The reference benchmark's own matrix on the engine:
BenchmarkReedSolomonErasureScheme (private/eestream/rs_test.go:553-634).

For RS(2,4), (20,50), (30,60), (50,80) and buffers of 100 B, 1 KiB, 256 KiB,
1 MiB, 5 MiB and 8 MiB (rounded down to a multiple of k, as the reference
does):
  Encode: ErasureScheme.Encode of the whole buffer (all n shares) -- ec_encode;
  Decode: ErasureScheme.Decode (Correct + Rebuild) of k+1+(i mod n/4) shares
          in shuffled order, as the reference's loop picks them -- ec_decode.
Both through the C-ABI with host buffers, synchronous: the ErasureScheme
boundary a Go caller would bind (PCIe and launch latency included).  Beside
each, the CPU oracle on one core (the reference's benchmark is one goroutine):
or_encode, and or_decode_fast (syndrome rows over whole buffers, as infectious'
Correct).  MB/s = the reference's SetBytes(dataSize) per call.  The crossover
is the smallest size from which the engine is faster.

Run on a GPU box:  python tools/bench_refmatrix.py [--json OUT] [--min-s 0.25]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from uplink_amd import _native  # noqa: E402
from oracle import oracle as O  # noqa: E402  (CPU baseline only)

CONFS = [(2, 4), (20, 50), (30, 60), (50, 80)]
SIZES = [100, 1 << 10, 256 << 10, 1 << 20, 5 << 20, 8 << 20]
ESS = 8 * 1024  # eestream.NewRSScheme(fec, 8*1024) in the benchmark; Encode/Decode ignore it


def size_name(b):
    if b > 10_000_000:
        return f"{b / (1 << 20):.0f}MB"
    if b > 1000:
        return f"{b / (1 << 10):.0f}KB"
    return f"{b}B"


def timeit(fn, min_s, min_iter=3, max_iter=2000):
    fn(0)  # warm (plans, workspaces, run-time encoders)
    ts = []
    t_end = time.perf_counter() + min_s
    i = 0
    while (i < min_iter or time.perf_counter() < t_end) and i < max_iter:
        t0 = time.perf_counter()
        fn(i)
        ts.append(time.perf_counter() - t0)
        i += 1
    return float(np.median(ts)), i


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    ap.add_argument("--min-s", type=float, default=0.25)
    ap.add_argument("--confs", default=None, help="e.g. 20,50;30,60")
    args = ap.parse_args()
    confs = CONFS if not args.confs else [tuple(int(x) for x in c.split(",")) for c in args.confs.split(";")]
    L = _native.load()
    oracle_lib = O.lib()
    u8p = ctypes.POINTER(ctypes.c_uint8)
    rng = np.random.default_rng(553)
    data = rng.integers(0, 256, 8 << 20, dtype=np.uint8)
    out = np.zeros(8 << 20, dtype=np.uint8)
    rows = []
    for k, n in confs:
        ctx = ctypes.c_void_p()
        rc = L.ec_create(k, n, ESS, ctypes.byref(ctx))
        assert rc == 0, _native.strerror(rc)
        L.ec_prepare_encoder(ctx, 1)
        f = O.FEC(k, n)
        enc = np.ascontiguousarray(f.enc, dtype=np.uint8)
        for exp_size in SIZES:
            ds = (exp_size // k) * k
            bs = ds // k
            src = data[:ds]
            shares = np.zeros((n, bs), dtype=np.uint8)
            assert L.ec_encode(ctx, src.ctypes.data, ds, shares.ctypes.data) == 0
            # the engine's shares are the oracle's (parity check of this very input)
            ref = np.zeros((n, bs), dtype=np.uint8)
            assert oracle_lib.or_encode(k, n, enc.ctypes.data_as(u8p), src.ctypes.data_as(u8p), ds,
                                        ref.ctypes.data_as(u8p)) == 0
            assert np.array_equal(shares, ref), f"RS({k},{n}) {ds} B: engine shares differ from the oracle"
            gpu_enc_out = np.zeros((n, bs), dtype=np.uint8)
            t_ge, it_ge = timeit(lambda i: L.ec_encode(ctx, src.ctypes.data, ds, gpu_enc_out.ctypes.data), args.min_s)
            cpu_out = np.zeros((n, bs), dtype=np.uint8)
            t_ce, it_ce = timeit(lambda i: oracle_lib.or_encode(k, n, enc.ctypes.data_as(u8p), src.ctypes.data_as(u8p),
                                                                 ds, cpu_out.ctypes.data_as(u8p)), args.min_s)
            # Decode: shuffled shares, k+1+(i mod n/4) of them (rs_test.go:617-625)
            order = np.arange(n)
            drng = np.random.default_rng(k * 7 + ds)
            perms = [drng.permutation(order) for _ in range(64)]

            def pick(i):
                m = min(k + 1 + i % (n // 4), n)
                return [int(x) for x in perms[i % 64][:m]]

            def gpu_dec(i):
                nums = pick(i)
                m = len(nums)
                carr = (ctypes.c_int * m)(*nums)
                parr = (ctypes.c_void_p * m)(*[shares[x].ctypes.data for x in nums])
                r = L.ec_decode(ctx, m, carr, parr, bs, out.ctypes.data)
                assert r == 0, _native.strerror(r)

            def cpu_dec(i):
                nums = pick(i)
                m = len(nums)
                carr = (ctypes.c_int * m)(*nums)
                parr = (u8p * m)(*[ref[x].ctypes.data_as(u8p) for x in nums])
                r = oracle_lib.or_decode_fast(k, n, enc.ctypes.data_as(u8p), m, carr, parr, bs,
                                              out.ctypes.data_as(u8p))
                assert r == 0, r

            gpu_dec(5)
            assert np.array_equal(out[:ds], src), f"RS({k},{n}) {ds} B: engine decode differs from the input"
            t_gd, it_gd = timeit(gpu_dec, args.min_s)
            t_cd, it_cd = timeit(cpu_dec, args.min_s)
            row = {"conf": f"r{k}t{n}", "k": k, "n": n, "size": size_name(ds), "bytes": ds,
                   "encode_gpu_us": t_ge * 1e6, "encode_cpu_us": t_ce * 1e6,
                   "decode_gpu_us": t_gd * 1e6, "decode_cpu_us": t_cd * 1e6,
                   "encode_gpu_MBps": ds / t_ge / 1e6, "encode_cpu_MBps": ds / t_ce / 1e6,
                   "decode_gpu_MBps": ds / t_gd / 1e6, "decode_cpu_MBps": ds / t_cd / 1e6,
                   "iters": [it_ge, it_ce, it_gd, it_cd]}
            rows.append(row)
            print(f"{row['conf']:>7} {row['size']:>6}  encode gpu {row['encode_gpu_us']:10.1f} us "
                  f"{row['encode_gpu_MBps']:9.1f} MB/s  cpu {row['encode_cpu_us']:10.1f} us {row['encode_cpu_MBps']:8.1f} MB/s"
                  f"  | decode gpu {row['decode_gpu_us']:10.1f} us {row['decode_gpu_MBps']:9.1f} MB/s  "
                  f"cpu {row['decode_cpu_us']:10.1f} us {row['decode_cpu_MBps']:8.1f} MB/s", flush=True)
        L.ec_destroy(ctx)
    cross = {}
    for k, n in confs:
        c = f"r{k}t{n}"
        mine = [r for r in rows if r["conf"] == c]
        for op in ("encode", "decode"):
            faster = [r["bytes"] for r in mine if r[f"{op}_gpu_us"] < r[f"{op}_cpu_us"]]
            # smallest size from which every larger size is faster on the engine
            x = None
            for r in reversed(mine):
                if r[f"{op}_gpu_us"] < r[f"{op}_cpu_us"]:
                    x = r["bytes"]
                else:
                    break
            cross[f"{c}/{op}"] = x if faster else None
    print(json.dumps({"crossover_bytes": cross}))
    if args.json:
        with open(args.json, "w") as fh:
            json.dump({"rows": rows, "crossover_bytes": cross, "cpu_threads": 1,
                       "boundary": "C-ABI host buffers (ec_encode / ec_decode), PCIe included"}, fh, indent=1)


if __name__ == "__main__":
    main()
