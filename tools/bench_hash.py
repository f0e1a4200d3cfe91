#!/usr/bin/env python3
"""Developer measurement for SURVEY.md §8f row 4 (piece hashing): BLAKE3 of
every piece of RS(29,80) 64 MiB segments (9040 stripes, pieces of
2,314,240 B), inputs resident in HBM.

Prints one JSON line:
  segment_hash   ec_hash_segments over NSEG segments: data pieces read in
                 place from the stripe-major segments (runs of 256 B), parity
                 pieces contiguous -- the upload path's form
  contiguous     ec_blake3_pieces over the same bytes laid out as [piece][len]
  roofline_valu  the hash is VALU-bound: each 64-byte block and each parent
                 node costs one compression (7 rounds x 8 G); peak = the
                 measured issue cost of the G instruction mix on 1024 SIMDs
  roofline_hbm   bytes hashed / time against the 8 TB/s HBM spec
  cpu_baseline   oracle/blake3_oracle.c (scalar C, one piece per thread) on a
                 bounded sample, on the host cores
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from uplink_amd import eestream, piecehash  # noqa: E402

K, N, ESS, STRIPES = 29, 80, 256, 9040
PLEN = STRIPES * ESS


def timed(fn, stream, iters):
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(stream):
        ev0.record(stream)
        for _ in range(iters):
            fn()
        ev1.record(stream)
    ev1.synchronize()
    return ev0.elapsed_time(ev1) / 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nseg", type=int, default=8)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--clock-ghz", type=float, default=2.4)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--cpu-sample-s", type=float, default=5.0)
    args = ap.parse_args()
    torch.cuda.set_device(0)
    sch = eestream.RSScheme(eestream.new_fec(K, N), ESS)
    codec = eestream.SegmentCodec(sch)
    nseg = args.nseg
    g = torch.Generator(device="cuda").manual_seed(1)
    segs = torch.randint(0, 256, (nseg, STRIPES * K * ESS), dtype=torch.uint8, device="cuda", generator=g)
    parity = torch.empty((nseg, N - K, PLEN), dtype=torch.uint8, device="cuda")
    codec.encode_segments(segs, nseg, STRIPES, parity, parity_only=True)
    pieces = torch.empty((nseg, N, PLEN), dtype=torch.uint8, device="cuda")
    codec.encode_segments(segs, nseg, STRIPES, pieces)
    h1 = torch.zeros((nseg, N, 32), dtype=torch.uint8, device="cuda")
    h2 = torch.zeros((nseg, N, 32), dtype=torch.uint8, device="cuda")
    st = torch.cuda.Stream()
    torch.cuda.synchronize()

    def seg_hash():
        piecehash.hash_segments(sch, segs, parity, nseg, STRIPES, h1, stream=st)

    def contig_hash():
        piecehash.blake3_device(pieces, nseg * N, PLEN, PLEN, h2, stream=st)

    for f in (seg_hash, contig_hash):  # warm up and settle clocks
        t_end = time.time() + 0.3
        while time.time() < t_end:
            f()
        torch.cuda.synchronize()
    t_seg = timed(seg_hash, st, args.iters)
    t_con = timed(contig_hash, st, args.iters)
    torch.cuda.synchronize()
    assert torch.equal(h1, h2), "segment-form and contiguous-form hashes differ"
    nbytes = nseg * N * PLEN
    out = {
        "metric": "blake3_piece_hash_GBps", "unit": "GB/s", "dtype": "u32",
        "config": {"workload": f"BLAKE3-256 of all {N} pieces of {nseg} RS({K},{N}) 64 MiB segments "
                               f"(pieces of {PLEN} B, resident in HBM)"},
        "bytes_per_launch": nbytes,
        "segment_hash": {"us_per_segment": t_seg / nseg * 1e6, "GBps": nbytes / t_seg / 1e9},
        "contiguous": {"us_per_segment": t_con / nseg * 1e6, "GBps": nbytes / t_con / 1e9},
    }
    out["roofline_hbm"] = {"achieved": out["segment_hash"]["GBps"], "peak": 8000.0, "unit": "GB/s",
                           "frac": out["segment_hash"]["GBps"] / 8000.0}
    # VALU issue roofline: one compression = 56 G, each 2 v_add3_u32 + 4 v_alignbit_b32 (4.2 cycles per
    # wave64 instruction on gfx950), 2 v_add_u32 (2.2) and 4 v_xor_b32 (2.4) -- tools/exp/op_probe.hip --
    # plus ~30 cycles of state set-up: ~2090 SIMD cycles per 64 lanes x 64 B.  Algorithmic compressions
    # per launch: one per 64-byte block plus one per parent node (chunks - 1 per piece).
    cyc = 56 * (2 * 4.2 + 4 * 4.2 + 2 * 2.2 + 4 * 2.4) + 30
    chunks = -(-PLEN // 1024)
    compressions = nseg * N * (PLEN // 64 + chunks - 1)
    peak = 256 * 4 * args.clock_ghz * 1e9 / cyc * 64  # compressions per second
    ach = compressions / t_seg
    out["roofline_valu"] = {"bound": "valu", "cycles_per_wave_compression": cyc, "achieved": ach / 1e9,
                            "peak": peak / 1e9, "unit": "G compressions/s", "frac": ach / peak}
    # CPU baseline: the scalar C oracle, one piece per thread, bounded sample
    from oracle import blake3 as ob
    host = pieces[0].cpu().numpy()
    done, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < args.cpu_sample_s:
        ob.blake3_many(host[:args.cpu_threads], threads=args.cpu_threads)
        done += args.cpu_threads
    dt = time.perf_counter() - t0
    out["cpu_baseline"] = {"value": done * PLEN / dt / 1e9, "unit": "GB/s", "cores": args.cpu_threads,
                           "kind": "port", "sample": f"{done} pieces of {PLEN} B in {dt:.1f} s"}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
