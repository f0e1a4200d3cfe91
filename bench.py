#!/usr/bin/env python3
"""Benchmark: GiB/s erasure encode+decode (device-resident), RS(29,80), 64 MiB segments.

BASELINE.json metric on configs[1]+configs[2], batched as
C4 (independent segments, sharded across ranks with no collective on the data
path: weak scaling).

One step on each rank = one batch of `--batch` (default 16) distinct synthetic
64 MiB segments (PadReader-padded to 9040 stripes x 29 x 256 B, stripe-major,
resident in HBM):
  1. ec_encode_segments: every segment -> 80 pieces of 2,314,240 B
     (segmentupload/encode.go:39-75 for all pieces at once), one launch;
  2. ec_rebuild_segments_batched: every segment rebuilt from exactly 29 pieces
     (stripe.go:382-428 for all stripes at once), one launch.  The 29-piece
     set cycles per step through {51..79} (all parity, worst case) and seven
     seeded random 29-subsets (default_rng(29)); decode plans are warmed in
     the untimed warm-up.
value = (payload bytes S_pad of all segments of all ranks) / (max over ranks
of the timed wall time) in GiB/s; S_pad is counted once per encode+decode
pair, i.e. value = S_pad / (t_encode + t_decode) aggregated.

Run: python bench.py [--gpus N --steps K --warmup W]; for N > 1 under
torch.distributed.run (one process per GPU).
"""
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
sys.path.insert(0, HERE)

from uplink_amd import _native  # noqa: E402

K, N, ESS = 29, 80, 256
RAW_SEGMENT = 64 * 1024 * 1024
STRIPE = K * ESS
NSTRIPES = (RAW_SEGMENT + 4 + STRIPE - 1) // STRIPE  # PadReader rule: 9040
S_PAD = NSTRIPES * STRIPE  # 67,112,960
PIECE = NSTRIPES * ESS  # 2,314,240
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--settle-s", type=float, default=0.3,
                    help="untimed steps run for at least this long before the W warm-up steps: the chip's clocks "
                         "ramp for tens of ms under sustained load (DESIGN.md §5)")
    ap.add_argument("--batch", type=int, default=16,
                    help="segments per step per GPU (12-16 measured best on MI355X, DESIGN.md §5)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-segments", type=int, default=4)
    ap.add_argument("--cpu-sample-s", type=float, default=10.0,
                    help="CPU baseline: cycle over the sample segments for at least this many seconds")
    ap.add_argument("--traffic-json", default=os.path.join(HERE, "profiles", "pmc_traffic.json"))
    return ap.parse_args()


def padded_segments(batch: int, seed: int, device) -> torch.Tensor:
    """batch distinct 64 MiB random segments + PadReader padding, on device."""
    g = torch.Generator(device=device)
    g.manual_seed(0x5EED0000 + seed)
    segs = torch.empty((batch, S_PAD), dtype=torch.uint8, device=device)
    segs[:, :RAW_SEGMENT] = torch.randint(0, 256, (batch, RAW_SEGMENT), dtype=torch.uint8, device=device,
                                          generator=g)
    p = S_PAD - RAW_SEGMENT
    segs[:, RAW_SEGMENT:] = p & 0xFF
    segs[:, -4:] = torch.tensor(list(p.to_bytes(4, "big")), dtype=torch.uint8, device=device)
    return segs


def share_sets():
    rng = np.random.default_rng(29)
    sets = [list(range(N - K, N))]
    for _ in range(7):
        sets.append(sorted(rng.choice(N, K, replace=False).tolist()))
    return sets


def cpu_baseline(threads: int, nseg: int, min_s: float):
    """Reference-shaped CPU loops of the oracle (per piece per stripe
    EncodeSingle, per stripe Rebuild with its k x k inversion) on `nseg`
    distinct segments, cycled until `min_s` seconds of CPU work: test
    infrastructure used only for this reported baseline."""
    from oracle import oracle as O
    f = O.FEC(K, N)
    rng = np.random.default_rng(7)
    segs = [np.frombuffer(rng.bytes(S_PAD), dtype=np.uint8) for _ in range(nseg)]
    sets = share_sets()
    t_enc = t_dec = 0.0
    done = 0
    while done < nseg or t_enc + t_dec < min_s:
        i = done
        seg = segs[i % nseg]
        done += 1
        t0 = time.perf_counter()
        pieces = f.encode_segment(seg, ESS, threads=threads)
        t1 = time.perf_counter()
        nums = sets[i % len(sets)]
        out = f.rebuild_segment(nums, [pieces[j] for j in nums], ESS, threads=threads)
        t2 = time.perf_counter()
        assert np.array_equal(out, seg)
        t_enc += t1 - t0
        t_dec += t2 - t1
    gib = done * S_PAD / 2**30
    return {
        "value": round(gib / (t_enc + t_dec), 4),
        "unit": "GiB/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{done} x 64 MiB RS(29,80) segments ({nseg} distinct, cycled): oracle reference-shaped encode "
                  f"(EncodeSingle per piece "
                  f"per stripe, AVX2 PSHUFB addmul) + per-stripe Rebuild from the same 29-piece sets as the GPU run; "
                  f"encode {t_enc:.3f}s, decode {t_dec:.3f}s wall on {threads} threads",
        "encode_gibps": round(gib / t_enc, 4),
        "decode_gibps": round(gib / t_dec, 4),
        "simd": ["scalar", "ssse3", "avx2"][O.lib().or_get_simd()],
    }


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # BENCH_DIST_BACKEND=gloo rehearses the N > 1 path on a one-GPU box (ranks share the
    # device, host-side collectives); the driver's multi-GPU runs use the default, RCCL.
    backend = os.environ.get("BENCH_DIST_BACKEND", "nccl")
    coll_dev = torch.device("cpu") if backend == "gloo" else None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local if backend != "gloo" else local % torch.cuda.device_count())
        if backend == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    L = _native.load()
    if L.ec_set_device(torch.cuda.current_device()) != 0:
        raise RuntimeError("ec_set_device failed")
    ctx = ctypes.c_void_p()
    rc = L.ec_create(K, N, ESS, ctypes.byref(ctx))
    if rc != 0:
        raise RuntimeError(f"ec_create failed: {_native.strerror(rc)}")

    B = args.batch
    segs = padded_segments(B, rank, dev)
    pieces = torch.empty((B, N, PIECE), dtype=torch.uint8, device=dev)
    out = torch.empty((B, S_PAD), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    sptr = stream.cuda_stream
    sets = share_sets()
    nums_c = [(ctypes.c_int * K)(*s) for s in sets]
    base = pieces.data_ptr()
    ptrs_c = [(ctypes.c_void_p * K)(*[base + j * PIECE for j in s]) for s in sets]

    def encode():
        r = L.ec_encode_segments(ctx, segs.data_ptr(), B, NSTRIPES, pieces.data_ptr(), 0, sptr)
        if r:
            raise RuntimeError(_native.strerror(r))

    def decode(step):
        i = step % len(sets)
        r = L.ec_rebuild_segments_batched(ctx, K, nums_c[i], ptrs_c[i], NSTRIPES, B, N * PIECE, S_PAD,
                                          out.data_ptr(), sptr)
        if r:
            raise RuntimeError(_native.strerror(r))

    def barrier():
        torch.cuda.synchronize(dev)
        if world > 1:
            import torch.distributed as dist
            dist.barrier()
        torch.cuda.synchronize(dev)

    # warm-up: every share set once (decode plans), then W steps
    for s in range(len(sets)):
        encode()
        decode(s)
    t_settle = time.perf_counter()
    s = 0
    while time.perf_counter() - t_settle < args.settle_s:
        encode()
        decode(s)
        s += 1
        if s % 8 == 0:
            torch.cuda.synchronize(dev)
    for s in range(args.warmup):
        encode()
        decode(s)
    barrier()

    # per-kernel HIP events on the launch stream (torch's current stream)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True),
           torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for s in range(args.steps):
        ev[s][0].record(stream)
        encode()
        ev[s][1].record(stream)
        decode(s)
        ev[s][2].record(stream)
    barrier()
    wall = time.perf_counter() - t0

    t_enc = sum(e[0].elapsed_time(e[1]) for e in ev) / args.steps * 1e-3  # s per launch
    t_dec = sum(e[1].elapsed_time(e[2]) for e in ev) / args.steps * 1e-3
    by_set = {}
    for st in range(args.steps):
        by_set.setdefault(st % len(sets), []).append(ev[st][1].elapsed_time(ev[st][2]) * 1e3 / B)
    if world > 1:
        import torch.distributed as dist
        tw = torch.tensor([wall], dtype=torch.float64, device=coll_dev or dev)
        dist.all_reduce(tw, op=dist.ReduceOp.MAX)
        wall = float(tw.item())

    # correctness of the last step (outside the timed region)
    verified = bool(torch.equal(out, segs))

    # informational, outside the timed region: the parity-only encode of BASELINE.md's table
    # (data pieces are the segment's own shares, served in place; the upload path uses this form)
    par = torch.empty((B, N - K, PIECE), dtype=torch.uint8, device=dev)
    pe = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for i in range(4):
        L.ec_encode_segments(ctx, segs.data_ptr(), B, NSTRIPES, par.data_ptr(), _native.EC_FLAG_PARITY_ONLY, sptr)
    pe[0].record(stream)
    for i in range(args.steps):
        if L.ec_encode_segments(ctx, segs.data_ptr(), B, NSTRIPES, par.data_ptr(), _native.EC_FLAG_PARITY_ONLY, sptr):
            raise RuntimeError("parity-only encode failed")
    pe[1].record(stream)
    pe[1].synchronize()
    t_par = pe[0].elapsed_time(pe[1]) / args.steps * 1e-3
    verified = verified and bool(torch.equal(par, pieces[:, K:]))
    del par
    if world > 1:
        import torch.distributed as dist
        v = torch.tensor([1 if verified else 0], device=coll_dev or dev)
        dist.all_reduce(v, op=dist.ReduceOp.MIN)
        verified = bool(v.item())

    total_payload = world * args.steps * B * S_PAD
    value = total_payload / 2**30 / wall
    enc_bytes = B * S_PAD * (1 + N / K)  # algorithmic bytes per encode launch
    dec_bytes = B * S_PAD * 2  # per decode launch
    enc_gbps = enc_bytes / t_enc / 1e9
    dec_gbps = dec_bytes / t_dec / 1e9
    kernels = {
        "encode": {"kernel": "rs_encode_special<29,80,4,4>", "avg_us": round(t_enc * 1e6, 2),
                   "bytes_per_launch": int(enc_bytes), "achieved_GBps": round(enc_gbps, 1)},
        "decode": {"kernel": "rs_matmul_jt<NW>", "avg_us": round(t_dec * 1e6, 2),
                   "bytes_per_launch": int(dec_bytes), "achieved_GBps": round(dec_gbps, 1),
                   "us_per_segment_by_set": {
                       f"set{i}:m={K - sum(1 for x in sets[i] if x < K)}": round(sum(v) / len(v), 2)
                       for i, v in sorted(by_set.items())}},
    }
    par_bytes = B * S_PAD * (1 + (N - K) / K)
    kernels["encode_parity_only"] = {
        "kernel": "rs_encode_special<29,80,8,4> (EC_FLAG_PARITY_ONLY)", "avg_us": round(t_par * 1e6, 2),
        "bytes_per_launch": int(par_bytes), "achieved_GBps": round(par_bytes / t_par / 1e9, 1),
        "frac": round(par_bytes / t_par / 1e9 / HBM_PEAK_GBPS, 4), "note": "informational, not in value"}
    dominant = "encode" if t_enc >= t_dec else "decode"
    dk = kernels[dominant]
    traffic = None
    try:
        with open(args.traffic_json) as fh:
            tj = json.load(fh)
        if tj.get("segments_per_launch", 8) == B:  # PMC bytes are per launch of this batch size
            traffic = tj.get(dominant, {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass
    line = {
        "metric": "GiB/s erasure encode+decode (device-resident), RS(29,80) 64 MiB segments",
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(wall / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (device-generated random segments, PadReader-padded)",
        "config": {"workload": "RS(29,80) encode+decode of 64 MiB segments (BASELINE configs[1]+[2], batched as "
                               "configs[3])", "k": K, "n": N, "erasure_share_size": ESS,
                   "segments_per_step_per_gpu": B, "stripes_per_segment": NSTRIPES,
                   "decode_share_sets": "cycle of {51..79} + 7 seeded random 29-subsets",
                   "parallelism": f"segments sharded over {world} GPU(s), no collective"},
        "roofline": {"bound": "hbm", "kernel": dominant, "achieved": round(dk["achieved_GBps"], 1),
                     "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": round(dk["achieved_GBps"] / HBM_PEAK_GBPS, 4),
                     "traffic": traffic},
        "kernels": kernels,
        "encode_gibps": round(B * S_PAD / 2**30 / t_enc, 2),
        "decode_gibps": round(B * S_PAD / 2**30 / t_dec, 2),
        "verified": verified,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        threads = min(os.cpu_count() or 1, 16)
        line["cpu_baseline"] = cpu_baseline(threads, args.cpu_sample_segments, args.cpu_sample_s)
    if rank == 0:
        print(json.dumps(line), flush=True)
    L.ec_destroy(ctx)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
