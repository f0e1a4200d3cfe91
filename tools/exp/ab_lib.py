"""Developer experiment (not product): A/B of library builds in ONE process,
in bench.py's own launch pattern (16 x 64 MiB RS(29,80) segments per launch,
each encode followed by a rebuild from a 29-piece set cycling through the
bench's 8 share sets), interleaved by rounds so box drift cancels
(cdna_hip_programming.md rule 24).  Per build: HIP-event time of every
encode and rebuild launch on the launch stream, and the parity-only encode
timed the same way; median and min over rounds.  Every build's pieces and
rebuilds are checked against the first build's.

  python tools/exp/ab_lib.py LIB_A LIB_B[@VAR=VALUE,...] ... [--rounds 6] [--pairs 8]
(VAR BODY=n is not an engine knob: ec_set_body(ctx, n) after ec_create.)
"""
from __future__ import annotations

import argparse
import ctypes
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from uplink_amd import _native  # noqa: E402

K, N, ESS, NSTRIPES, S_PAD, PIECE = bench.K, bench.N, bench.ESS, bench.NSTRIPES, bench.S_PAD, bench.PIECE


def load(path):
    lib = ctypes.CDLL(os.path.abspath(path))
    for name, (res, args) in _native.SIGNATURES.items():
        if hasattr(lib, name):
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
    return lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--pairs", type=int, default=8, help="encode+rebuild launch pairs per round and build")
    ap.add_argument("--batch", type=int, default=16)
    args = ap.parse_args()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    B = args.batch
    stream = torch.cuda.current_stream(dev)
    sptr = stream.cuda_stream
    segs = bench.padded_segments(B, 1, dev)
    pieces = torch.empty((B, N, PIECE), dtype=torch.uint8, device=dev)
    outs = torch.empty((B, S_PAD), dtype=torch.uint8, device=dev)
    par = torch.empty((B, N - K, PIECE), dtype=torch.uint8, device=dev)
    sets = bench.share_sets()
    nums_c = [(ctypes.c_int * K)(*s) for s in sets]
    ptrs_c = [(ctypes.c_void_p * K)(*[pieces.data_ptr() + j * PIECE for j in s]) for s in sets]
    builds = []
    ref = None
    for spec in args.libs:
        # LIB[@VAR=VALUE,...]: environment set while the context is created (engine knobs read at ec_create)
        p, _, envs = spec.partition("@")
        saved = {}
        for kv in filter(None, envs.split(",")):
            var, _, val = kv.partition("=")
            saved[var] = os.environ.get(var)
            os.environ[var] = val
        L = load(p)
        ctx = ctypes.c_void_p()
        assert L.ec_create(K, N, ESS, ctypes.byref(ctx)) == 0
        if "BODY" in saved:  # BODY=n: ec_set_body(ctx, n) (2 = straight-line: the SL encode for any (k, n))
            assert L.ec_set_body(ctx, int(os.environ["BODY"])) == 0
        for var, val in saved.items():
            if val is None:
                os.environ.pop(var)
            else:
                os.environ[var] = val
        tag = os.path.basename(os.path.dirname(os.path.abspath(p))) + (f"@{envs}" if envs else "")
        pieces.zero_()
        assert L.ec_encode_segments(ctx, segs.data_ptr(), B, NSTRIPES, pieces.data_ptr(), 0, sptr) == 0
        torch.cuda.synchronize()
        if ref is None:
            ref = pieces.clone()
        ok = bool(torch.equal(pieces, ref))
        for i in range(len(sets)):  # decode plans (and their generated code) made here, outputs checked
            for _ in range(2):
                outs.zero_()
                assert L.ec_rebuild_segments_batched(ctx, K, nums_c[i], ptrs_c[i], NSTRIPES, B, N * PIECE, S_PAD,
                                                     outs.data_ptr(), sptr) == 0
            torch.cuda.synchronize()
            ok = ok and bool(torch.equal(outs, segs))
        par.zero_()
        assert L.ec_encode_segments(ctx, segs.data_ptr(), B, NSTRIPES, par.data_ptr(), _native.EC_FLAG_PARITY_ONLY,
                                    sptr) == 0
        torch.cuda.synchronize()
        ok = ok and bool(torch.equal(par, ref[:, K:]))
        bid = L.ec_build_id().decode() if hasattr(L, "ec_build_id") else "?"
        print(f"{tag:24s} build {bid} results {'match' if ok else 'DIFFER'}", flush=True)
        builds.append((tag, L, ctx))
    counter = [0]
    per_set = {}  # library -> share set -> rebuild us per launch

    def run(L, ctx, flags):
        evs = []
        for _ in range(args.pairs):
            i = counter[0] % len(sets)
            counter[0] += 1
            e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            e[0].record(stream)
            dst = par if flags else pieces
            assert L.ec_encode_segments(ctx, segs.data_ptr(), B, NSTRIPES, dst.data_ptr(), flags, sptr) == 0
            e[1].record(stream)
            assert L.ec_rebuild_segments_batched(ctx, K, nums_c[i], ptrs_c[i], NSTRIPES, B, N * PIECE, S_PAD,
                                                 outs.data_ptr(), sptr) == 0
            e[2].record(stream)
            evs.append((e, i))
        torch.cuda.synchronize()
        enc = sum(e[0].elapsed_time(e[1]) for e, _ in evs) / len(evs) * 1e3
        dec = sum(e[1].elapsed_time(e[2]) for e, _ in evs) / len(evs) * 1e3
        if not flags:
            for e, i in evs:
                per_set.setdefault(L, {}).setdefault(i, []).append(e[1].elapsed_time(e[2]) * 1e3)
        return enc, dec

    t0 = time.perf_counter()  # settle the clocks
    while time.perf_counter() - t0 < 0.5:
        run(builds[0][1], builds[0][2], 0)
    res = {tag: {"enc": [], "dec": [], "par": []} for tag, _, _ in builds}
    for r in range(args.rounds):
        order = builds if r % 2 == 0 else builds[::-1]
        for tag, L, ctx in order:
            e, d = run(L, ctx, 0)
            p, _ = run(L, ctx, _native.EC_FLAG_PARITY_ONLY)
            res[tag]["enc"].append(e)
            res[tag]["dec"].append(d)
            res[tag]["par"].append(p)
    eb, db, pb = B * S_PAD * (1 + N / K), 2 * B * S_PAD, B * S_PAD * (1 + (N - K) / K)
    print(f"us per launch of {B} segments, median (min) over {args.rounds} rounds x {args.pairs} pairs; "
          f"frac of 8 TB/s")
    for tag, v in res.items():
        def md(x):
            return sorted(x)[len(x) // 2]
        e, d, p = md(v["enc"]), md(v["dec"]), md(v["par"])
        print(f"{tag:24s} encode {e:7.1f} ({min(v['enc']):7.1f}) {eb / e / 8e6:.4f}   rebuild {d:6.1f} "
              f"({min(v['dec']):6.1f}) {db / d / 8e6:.4f}   parity-only {p:6.1f} ({min(v['par']):6.1f}) "
              f"{pb / p / 8e6:.4f}", flush=True)
    print("rebuild us per launch by share set (m = missing data shares), median over the run")
    for tag, L, _ in builds:
        row = []
        for i, v in sorted(per_set.get(L, {}).items()):
            m = K - sum(1 for x in sets[i] if x < K)
            row.append(f"m={m}:{sorted(v)[len(v) // 2]:.1f}")
        print(f"{tag:24s} " + " ".join(row), flush=True)


if __name__ == "__main__":
    main()
