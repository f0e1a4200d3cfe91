#!/usr/bin/env python3
"""Benchmark: GiB/s erasure encode+decode (device-resident), RS(29,80), 64 MiB segments.

BASELINE.json metric on configs[1]+configs[2], run as
configs[3]: a batch of --total-segments (default 1024) independent 64 MiB
segments, sharded contiguously over the ranks (uplink_amd/shard.py:
128 per GPU at 8 GPUs) with no collective on the data path.

One step = every rank processes its whole shard once, in launches of
`--batch` (default 32) segments, each launch pair being
  1. ec_encode_segments: 32 segments -> 80 pieces of 2,314,240 B each
     (segmentupload/encode.go:39-75 for all pieces at once);
  2. ec_rebuild_segments_sets: the 32 segments rebuilt, each from exactly 29
     of its pieces in a share set of its own -- the way uplink downloads: every
     segment from whichever 29 pieces answered first (stripe.go:314-354), one
     GetWithOptions per segment (client.go:273-308).  Every timed launch gets
     32 fresh seeded 29-subsets (every step's first segment from the
     all-parity {51..79}, the worst case); no decode plan is made or warmed
     (the decode rows are solved on the GPU inside the call, rs_sets.hip).
The segments are synthetic (device-generated random bytes, PadReader-padded to
9040 stripes x 29 x 256 B), from a pool of 2 x 32 distinct segments per rank
cycled over the shard: 1024 segments' pieces would not fit one GPU (SURVEY §8d
C4).  value = (payload bytes S_pad of all segments of all ranks, all steps) /
(max over ranks of the timed wall time) in GiB/s, i.e. S_pad / (t_encode +
t_decode) aggregated; the total is fixed, so scaling is "strong".

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
from uplink_amd.shard import segment_seed, shard_range  # noqa: E402

K, N, ESS = 29, 80, 256
RAW_SEGMENT = 64 * 1024 * 1024
STRIPE = K * ESS
NSTRIPES = (RAW_SEGMENT + 4 + STRIPE - 1) // STRIPE  # PadReader rule: 9040
S_PAD = NSTRIPES * STRIPE  # 67,112,960
PIECE = NSTRIPES * ESS  # 2,314,240
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec


# the library's RS(29,80) encoders as rocprofv3 names them (rs_encoder.hpp: 8 compute + 4
# loader waves; the last argument tells the full encode from the parity-only one)
ENC_FULL_KERNEL = "rs_encode_special<29, 80, 8, 4, true>"
ENC_PARITY_KERNEL = "rs_encode_special<29, 80, 8, 4, false>"

def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--settle-s", type=float, default=0.3,
                    help="untimed launches run for at least this long before the W warm-up steps: the chip's clocks "
                         "ramp for tens of ms under sustained load (DESIGN.md §5)")
    ap.add_argument("--total-segments", type=int, default=1024,
                    help="BASELINE configs[3]: segments per step over all ranks (sharded contiguously)")
    ap.add_argument("--batch", type=int, default=32,
                    help="segments per launch (32: +1.3 %% over 16, the rebuild's grid twice as long; DESIGN.md §5)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-other-configs", action="store_true",
                    help="skip the RS(20,50)/(30,60)/(50,80) entries (PMC passes: only RS(29,80) launches)")
    ap.add_argument("--cpu-sample-s", type=float, default=10.0,
                    help="CPU baseline: seconds of reference-shaped work on all host cores (plus shorter single-core "
                         "and optimised-variant samples)")
    ap.add_argument("--body", choices=["auto", "jump-table", "straight-line"], default="auto",
                    help="ec_set_body for the bench's context (include/uplink_ec.h); default: the library's choice")
    ap.add_argument("--lib", default=None, help="another build of libuplink_ec.so (A/B runs of library variants)")
    ap.add_argument("--traffic-json", default=os.path.join(HERE, "profiles", "pmc_traffic.json"))
    return ap.parse_args()


def padded_segments(batch: int, seed: int, device) -> torch.Tensor:
    """batch distinct 64 MiB random segments + PadReader padding, on device."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
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


def fresh_launch_sets(seed: int, nb: int, all_parity_first: bool):
    """The share sets of one timed decode launch: nb fresh seeded 29-subsets,
    with all_parity_first the first of them the all-parity {51..79} (the
    worst case: 29 rows to compute)."""
    rng = np.random.default_rng(seed)
    sets = [sorted(int(x) for x in rng.permutation(N)[:K]) for _ in range(nb)]
    if all_parity_first:
        sets[0] = list(range(N - K, N))
    return sets


def cgroup_cpus():
    """CPUs the cgroup quota grants this process (cgroup v2 cpu.max or v1
    cfs quota), or None when unlimited / unknown."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, p = fh.read().split()[:2]
            if q != "max":
                return max(1, int(int(q) / int(p)))
            return None
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as fh:
            q = int(fh.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as fh:
            p = int(fh.read())
        return max(1, q // p) if q > 0 else None
    except (OSError, ValueError):
        return None


def host_cpus():
    """The cores this process may run on -- its affinity set, capped by a
    cgroup CPU quota when there is one -- and what they are (logged with the
    baseline)."""
    affinity = len(os.sched_getaffinity(0))
    quota = cgroup_cpus()
    cores = min(affinity, quota) if quota else affinity
    model = ""
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return cores, os.cpu_count() or cores, model, affinity, quota


def cpu_baseline(min_s: float):
    """The oracle's CPU loops on the GPU box's host (test infrastructure, used
    only for this reported baseline):
      * reference shape (the headline figure): per piece per stripe
        EncodeSingle, per stripe Rebuild with its k x k inversion -- what Go
        eestream does -- on all cores of this process's CPU set, for >= min_s;
      * the same on one core;
      * the optimised variant: all rows per block of stripes, one inversion per
        share set, all cores."""
    from oracle import oracle as O
    f = O.FEC(K, N)
    rng = np.random.default_rng(7)
    nseg = 4
    segs = [np.frombuffer(rng.bytes(S_PAD), dtype=np.uint8) for _ in range(nseg)]
    sets = share_sets()
    cores, nproc, model, affinity, quota = host_cpus()

    def run(threads, limit_s, fast=False, min_segs=1):
        t_enc = t_dec = 0.0
        done = 0
        while done < min_segs or t_enc + t_dec < limit_s:
            seg = segs[done % nseg]
            nums = sets[done % len(sets)]
            t0 = time.perf_counter()
            pieces = (f.fast_encode_segment if fast else f.encode_segment)(seg, ESS, threads=threads)
            t1 = time.perf_counter()
            out = (f.fast_rebuild_segment if fast else f.rebuild_segment)(nums, [pieces[j] for j in nums], ESS,
                                                                          threads=threads)
            t2 = time.perf_counter()
            assert np.array_equal(out, seg)
            t_enc += t1 - t0
            t_dec += t2 - t1
            done += 1
        gib = done * S_PAD / 2**30
        return {"value": round(gib / (t_enc + t_dec), 4), "encode_gibps": round(gib / t_enc, 4),
                "decode_gibps": round(gib / t_dec, 4), "segments": done, "encode_s": round(t_enc, 3),
                "decode_s": round(t_dec, 3)}

    ref = run(cores, min_s, min_segs=nseg)
    one = run(1, min_s / 3)
    fast = run(cores, min_s / 2, fast=True, min_segs=nseg)
    return {
        "value": ref["value"],
        "unit": "GiB/s",
        "cores": cores,
        "kind": "port",
        "sample": f"{ref['segments']} x 64 MiB RS(29,80) segments ({nseg} distinct, cycled): oracle reference-shaped "
                  f"encode (EncodeSingle per piece per stripe, AVX2 PSHUFB addmul) + per-stripe Rebuild from the same "
                  f"29-piece sets as the GPU run; encode {ref['encode_s']}s, decode {ref['decode_s']}s wall on {cores} "
                  f"threads (this process's CPUs: affinity {affinity}, cgroup quota {quota or 'none'}; nproc {nproc}; "
                  f"{model})",
        "encode_gibps": ref["encode_gibps"],
        "decode_gibps": ref["decode_gibps"],
        "single_core": {"value": one["value"], "encode_gibps": one["encode_gibps"],
                        "decode_gibps": one["decode_gibps"], "segments": one["segments"]},
        "optimised_all_cores": {"value": fast["value"], "encode_gibps": fast["encode_gibps"],
                                "decode_gibps": fast["decode_gibps"], "segments": fast["segments"],
                                "what": "all rows per block of 32 stripes, one inversion per share set"},
        "simd": ["scalar", "ssse3", "avx2"][O.lib().or_get_simd()],
    }


def oracle_spot_check(pieces_seg0: torch.Tensor, seg0: torch.Tensor, stripes: int = 64) -> bool:
    """The first `stripes` stripes of one segment's pieces, against the oracle
    (outside the timed region; the rebuild check alone would also pass a
    wrong-but-self-consistent encoder)."""
    from oracle import oracle as O
    seg = seg0[: stripes * STRIPE].cpu().numpy()
    ref = O.FEC(K, N).encode_segment(seg, ESS, threads=4)
    got = pieces_seg0[:, : stripes * ESS].cpu().numpy()
    return bool(np.array_equal(got, ref))


def other_configs(L, dev, sptr, reps: int = 10):
    """Informational, outside the timed region: the reference benchmark's
    other configurations (private/eestream/rs_test.go:553-634: RS(20,50),
    (30,60), (50,80)) on 8 x 64 MiB segments -- encode of all pieces and
    rebuild from the last k pieces (all parity), HIP-event times per launch
    and the HBM roofline fraction of each."""
    out = {}
    nseg = 8
    for k, n in ((20, 50), (30, 60), (50, 80)):
        stripe = k * ESS
        nstripes = (RAW_SEGMENT + 4 + stripe - 1) // stripe
        spad, plen = nstripes * stripe, nstripes * ESS
        ctx = ctypes.c_void_p()
        if L.ec_create(k, n, ESS, ctypes.byref(ctx)):
            continue
        segs = torch.randint(0, 256, (nseg, spad), dtype=torch.uint8, device=dev)
        pcs = torch.empty((nseg, n, plen), dtype=torch.uint8, device=dev)
        back = torch.empty((nseg, spad), dtype=torch.uint8, device=dev)
        nums = (ctypes.c_int * k)(*range(n - k, n))
        ptrs = (ctypes.c_void_p * k)(*[pcs.data_ptr() + j * plen for j in range(n - k, n)])

        def enc():
            assert L.ec_encode_segments(ctx, segs.data_ptr(), nseg, nstripes, pcs.data_ptr(), 0, sptr) == 0

        def dec():
            assert L.ec_rebuild_segments_batched(ctx, k, nums, ptrs, nstripes, nseg, n * plen, spad, back.data_ptr(),
                                                 sptr) == 0
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        for _ in range(3):
            enc()
            dec()
        # the set's straight-line code is made in the background after its first launch: wait for it,
        # so the timed rebuilds are the warm ones (as the headline's sets are)
        L.ec_prepare_rebuild(ctx, k, nums, 1)
        ev[0].record()
        for _ in range(reps):
            enc()
        ev[1].record()
        for _ in range(reps):
            dec()
        ev[2].record()
        ev[2].synchronize()
        t_e = ev[0].elapsed_time(ev[1]) / reps * 1e-3
        t_d = ev[1].elapsed_time(ev[2]) / reps * 1e-3
        eb, db = nseg * spad * (1 + n / k), nseg * spad * 2
        out[f"RS({k},{n})"] = {
            "encode_kernel": L.ec_encode_kernel_name(ctx).decode(),
            "encode_us_per_segment": round(t_e / nseg * 1e6, 2), "encode_GBps": round(eb / t_e / 1e9, 1),
            "encode_frac": round(eb / t_e / 1e9 / HBM_PEAK_GBPS, 4),
            "rebuild_all_parity_us_per_segment": round(t_d / nseg * 1e6, 2), "rebuild_GBps": round(db / t_d / 1e9, 1),
            "rebuild_frac": round(db / t_d / 1e9 / HBM_PEAK_GBPS, 4),
            "verified": bool(torch.equal(back, segs))}
        del segs, pcs, back
        L.ec_destroy(ctx)
    return out


def decode_with_detection(L, dev, sptr, reps: int = 4, nb: int = 16, extras=(1, 4, 10, 20)):
    """Informational, outside the timed region: Decode with error detection on
    whole RS(29,80) 64 MiB segments, nb per call (ec_decode_segments_batched:
    syndrome rows checked for zero in the kernel, then Rebuild) from
    k+1 .. k+n/4 clean shares in shuffled order, the reference benchmark's
    Decode shape (private/eestream/rs_test.go:616-631) at segment size.  Per
    extra-share count: wall time per segment (synchronous: the check's outcome
    is read back) and HBM fraction of the algorithmic bytes (the ns pieces
    read + the segment written)."""
    ctx = ctypes.c_void_p()
    if L.ec_create(K, N, ESS, ctypes.byref(ctx)):
        return {}
    nstripes = (RAW_SEGMENT + 4 + K * ESS - 1) // (K * ESS)
    spad, plen = nstripes * K * ESS, nstripes * ESS
    segs = torch.randint(0, 256, (nb, spad), dtype=torch.uint8, device=dev)
    pcs = torch.empty((nb, N, plen), dtype=torch.uint8, device=dev)
    assert L.ec_encode_segments(ctx, segs.data_ptr(), nb, nstripes, pcs.data_ptr(), 0, sptr) == 0
    back = torch.empty_like(segs)
    rng = np.random.default_rng(616)
    res = {}
    ok = True
    for extra in extras:
        sets = [[int(x) for x in rng.permutation(N)[:K + extra]] for _ in range(4)]
        args = [((ctypes.c_int * len(s))(*s), (ctypes.c_void_p * len(s))(*[pcs.data_ptr() + i * plen for i in s]))
                for s in sets]

        def call(i):
            nums, ptrs = args[i % len(args)]
            rc = L.ec_decode_segments_batched(ctx, K + extra, nums, ptrs, nstripes, nb, N * plen, spad,
                                              back.data_ptr(), sptr)
            assert rc == 0, _native.strerror(rc)
        for i in range(2 * len(args)):  # plans made (and their generated code: second use), outputs checked
            back.fill_(0)
            call(i)
            torch.cuda.synchronize()
            ok = ok and bool(torch.equal(back, segs))
        torch.cuda.synchronize()
        walls = []  # per call (each returns synchronised: the check's outcome is read back)
        for i in range(reps * len(args)):
            t0 = time.perf_counter()
            call(i)
            walls.append((time.perf_counter() - t0) / nb)
        wall = sum(walls) / len(walls)
        alg = plen * (K + extra) + spad
        res[f"k+{extra}"] = {"us_per_segment": round(wall * 1e6, 2), "GBps": round(alg / wall / 1e9, 1),
                             "frac": round(alg / wall / 1e9 / HBM_PEAK_GBPS, 4),
                             "data_GiBps": round(spad / wall / 2**30, 1),
                             "us_per_segment_median_call": round(float(np.median(walls)) * 1e6, 2),
                             "us_per_segment_max_call": round(max(walls) * 1e6, 2)}
    res["verified"] = ok
    res["note"] = (f"clean shares, {nb} segments per call, wall clock per call (launch, check read-back and sync "
                   "included), mean (and median, max) over the calls; 4 seeded share sets per count, plans warm; "
                   "informational, not in value")
    del segs, pcs, back
    L.ec_destroy(ctx)
    return res


def fresh_share_sets(L, dev, sptr, nb: int = 16, launches: int = 12):
    """Informational, outside the timed region: the rebuild when every launch
    comes with a share set the context has not seen (a real download: each
    segment's pieces come from whichever 29 nodes answered first, so its
    decode plan is new) -- plan creation (inversion, generated code, module
    load, tables) included, wall clock per launch, synchronous, after the
    64-plan cache is full.  Against the same launches with warm plans."""
    ctx = ctypes.c_void_p()
    if L.ec_create(K, N, ESS, ctypes.byref(ctx)):
        return {}
    nstripes = (RAW_SEGMENT + 4 + K * ESS - 1) // (K * ESS)
    spad, plen = nstripes * K * ESS, nstripes * ESS
    segs = torch.randint(0, 256, (nb, spad), dtype=torch.uint8, device=dev)
    pcs = torch.empty((nb, N, plen), dtype=torch.uint8, device=dev)
    assert L.ec_encode_segments(ctx, segs.data_ptr(), nb, nstripes, pcs.data_ptr(), 0, sptr) == 0
    back = torch.empty_like(segs)
    rng = np.random.default_rng(64)

    def subset():  # 16..29 missing data shares, as bench.py's random sets
        return sorted(int(x) for x in rng.permutation(N)[:K])

    def run(nums, n):
        cn = (ctypes.c_int * K)(*nums)
        cp = (ctypes.c_void_p * K)(*[pcs.data_ptr() + i * plen for i in nums])
        assert L.ec_rebuild_segments_batched(ctx, K, cn, cp, nstripes, n, N * plen, spad, back.data_ptr(), sptr) == 0
    for _ in range(70):  # fill the plan cache past its 64 entries
        run(subset(), 1)
    torch.cuda.synchronize()
    res = {}
    for n in (1, nb):
        sets = [subset() for _ in range(launches)]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for s in sets:
            run(s, n)
            torch.cuda.synchronize()
        fresh = (time.perf_counter() - t0) / launches
        t0 = time.perf_counter()
        for s in sets:  # the same sets again (their generated code is being made in the background)
            run(s, n)
            torch.cuda.synchronize()
        second = (time.perf_counter() - t0) / launches
        for s in sets:  # (wait for the background builder: the warm launches run the generated code)
            L.ec_prepare_rebuild(ctx, K, (ctypes.c_int * K)(*s), 1)
        t0 = time.perf_counter()
        for s in sets:  # and once more: plans and code warm
            run(s, n)
            torch.cuda.synchronize()
        warm = (time.perf_counter() - t0) / launches
        res[f"{n} segment(s) per launch"] = {"first_launch_us": round(fresh * 1e6, 1),
                                             "second_launch_us": round(second * 1e6, 1),
                                             "warm_launch_us": round(warm * 1e6, 1)}
    res["note"] = ("ec_rebuild_segments_batched, EC_BODY_AUTO: a share set without generated code runs the "
                   "share-set pass (decode rows solved on the GPU, jump-table body) and has its straight-line code "
                   "made in the background; warm = after ec_prepare_rebuild(wait)")
    del segs, pcs, back
    L.ec_destroy(ctx)
    return res


def _r(x, nd):
    return None if x is None else round(x, nd)


def _ratio(a, b):
    return None if not b else round(a / b, 4)


def on_box_ceilings(L, dev, stream, read_bytes: int = 1 << 30, reps: int = 10):
    """GB/s (bytes read + written) of the library's streaming probe kernels in each
    kernel's read:write mix, on this box, now (include/uplink_ec.h ec_bw_probe)."""
    src = torch.randint(0, 256, (read_bytes,), dtype=torch.uint8, device=dev)
    dst = torch.empty(read_bytes * 11 // 4 + 4096, dtype=torch.uint8, device=dev)
    out = {}
    for name, shape in (("copy", _native.EC_PROBE_COPY), ("encode_mix", _native.EC_PROBE_ENCODE_MIX),
                        ("parity_mix", _native.EC_PROBE_PARITY_MIX)):
        moved = ctypes.c_size_t()
        for _ in range(3):
            if L.ec_bw_probe(shape, src.data_ptr(), read_bytes, dst.data_ptr(), ctypes.byref(moved),
                             stream.cuda_stream):
                raise RuntimeError("ec_bw_probe failed")
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
        ev[0].record(stream)
        for i in range(reps):
            L.ec_bw_probe(shape, src.data_ptr(), read_bytes, dst.data_ptr(), ctypes.byref(moved), stream.cuda_stream)
            ev[i + 1].record(stream)
        ev[-1].synchronize()
        t = float(np.median([ev[i].elapsed_time(ev[i + 1]) * 1e-3 for i in range(reps)]))
        out[name] = moved.value / t / 1e9
    del src, dst
    return out


def fresh_sets_leg(L, ctx, dev, sptr, nb: int = 32, reps: int = 16):
    """The decode the way uplink runs it: every segment of a
    download is rebuilt from whichever 29 pieces answered first
    (private/eestream/stripe.go:314-354), so each brings a share set of its own
    (ec_rebuild_segments_sets: the decode rows solved on the GPU, stream-ordered,
    jump-table body).  Outside the timed region, informational:
      * "32 segments, 32 fresh seeded 29-subsets per launch": HIP-event time per
        call, calls back to back, and its HBM fraction (2 x S_pad per segment);
      * "one segment, fresh set": wall clock per call, from the call to its
        stream synchronised (median), and the stream time of such calls back
        to back."""
    rng = np.random.default_rng(3229)
    segs = torch.randint(0, 256, (nb, S_PAD), dtype=torch.uint8, device=dev)
    pcs = torch.empty((nb, N, PIECE), dtype=torch.uint8, device=dev)
    outs = torch.empty_like(segs)
    stream = torch.cuda.current_stream(dev)
    if L.ec_encode_segments(ctx, segs.data_ptr(), nb, NSTRIPES, pcs.data_ptr(), 0, sptr):
        raise RuntimeError("encode failed")

    def fresh(count):
        return [sorted(int(x) for x in rng.permutation(N)[:K]) for _ in range(count)]

    def prep(sets):  # the call's arrays, made before the timed calls (a Go caller holds its slices)
        n = len(sets)
        flat = [x for st in sets for x in st]
        return (n, (ctypes.c_int * n)(*[K] * n), (ctypes.c_int * len(flat))(*flat),
                (ctypes.c_void_p * len(flat))(*[pcs[g].data_ptr() + x * PIECE for g, st in enumerate(sets) for x in st]),
                (ctypes.c_void_p * n)(*[outs[g].data_ptr() for g in range(n)]))

    def go(a):
        n, nsh, nums, ptrs, optr = a
        rc = L.ec_rebuild_segments_sets(ctx, n, nsh, nums, ptrs, NSTRIPES, optr, sptr)
        if rc:
            raise RuntimeError(_native.strerror(rc))

    def call(sets):
        go(prep(sets))
    outs.zero_()
    call(fresh(nb))
    torch.cuda.synchronize(dev)
    ok = bool(torch.equal(outs, segs))
    all_sets = [fresh(nb) for _ in range(reps)]
    all_args = [prep(x) for x in all_sets]
    # clock settle at the timed loop's duty cycle (calls back to back, arrays made
    # beforehand): a settle loop that builds its arrays in Python leaves the GPU idle
    # between calls, and the first timed calls then run at a clock the steady state
    # does not keep (816-838 us, then 930-1150, profiles/r05/h)
    t_end = time.perf_counter() + 0.3
    i = 0
    while time.perf_counter() < t_end:
        go(all_args[i % reps])
        i += 1
    torch.cuda.synchronize(dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
    ev[0].record(stream)
    for i in range(reps):
        go(all_args[i])
        ev[i + 1].record(stream)
    ev[-1].synchronize()
    per = [ev[i].elapsed_time(ev[i + 1]) * 1e-3 for i in range(reps)]
    t = float(np.median(per))
    ms = sorted(sum(1 for x in st if x >= K) for st in all_sets[0])
    batch = {"us_per_launch": round(t * 1e6, 1), "us_per_segment": round(t / nb * 1e6, 2),
             "GBps": round(2 * S_PAD * nb / t / 1e9, 1), "frac": round(2 * S_PAD * nb / t / 1e9 / HBM_PEAK_GBPS, 4),
             "rows_per_segment": f"{ms[0]}..{ms[-1]} (median {ms[len(ms) // 2]})", "verified": ok}
    walls = []
    for _ in range(4 * reps):
        one = prep(fresh(1))
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        go(one)
        stream.synchronize()  # (the caller's stream, as a Go caller waits for its own call: hipStreamSynchronize)
        walls.append(time.perf_counter() - t0)
    singles = [prep(fresh(1)) for _ in range(reps)]
    torch.cuda.synchronize(dev)
    e2 = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    e2[0].record(stream)
    for one in singles:
        go(one)
    e2[1].record(stream)
    e2[1].synchronize()
    b2b = e2[0].elapsed_time(e2[1]) * 1e-3 / reps
    single = {"wall_us_median": round(float(np.median(walls)) * 1e6, 1), "wall_us_min": round(min(walls) * 1e6, 1),
              "stream_us_back_to_back": round(b2b * 1e6, 1),
              "frac_back_to_back": round(2 * S_PAD / b2b / 1e9 / HBM_PEAK_GBPS, 4)}
    del segs, pcs, outs
    return {f"{nb} segments, {nb} fresh seeded 29-subsets per launch": batch, "one segment, fresh set": single,
            "note": "ec_rebuild_segments_sets; outside the timed region, informational, not in value"}


def warm_shared_set_leg(L, ctx, encode, pieces, outs, segs, pool, B, dev, stream, sptr, rounds: int = 2):
    """Informational, outside the timed region: the decode from ONE share set
    per launch with its plan warm (ec_rebuild_segments_batched; the cycle of
    {51..79} + 7 seeded random 29-subsets, each set's straight-line code made
    and waited for first) -- what a caller that keeps reusing a set gets.
    Timed as the headline decode: each decode launch right after an encode."""
    sets = share_sets()
    nums_c = [(ctypes.c_int * K)(*s) for s in sets]
    ptrs_c = [[(ctypes.c_void_p * K)(*[p.data_ptr() + j * PIECE for j in s]) for s in sets] for p in pieces]

    def dec(slot, i):
        r = L.ec_rebuild_segments_batched(ctx, K, nums_c[i], ptrs_c[slot][i], NSTRIPES, B, N * PIECE, S_PAD,
                                          outs[slot].data_ptr(), sptr)
        if r:
            raise RuntimeError(_native.strerror(r))
    for slot in range(pool):
        for i in range(len(sets)):
            encode(slot, B)
            dec(slot, i)
    for st in sets:  # the sets' generated code, made in the background, ready before timing
        L.ec_prepare_rebuild(ctx, K, (ctypes.c_int * K)(*st), 1)
    t_settle = time.perf_counter()
    j = 0
    while time.perf_counter() - t_settle < 0.3:
        encode(j % pool, B)
        dec(j % pool, j % len(sets))
        j += 1
        torch.cuda.synchronize(dev)
    ev = []
    for r in range(rounds * len(sets)):
        slot, i = r % pool, r % len(sets)
        e = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        encode(slot, B)
        e[0].record(stream)
        dec(slot, i)
        e[1].record(stream)
        ev.append((e, i))
    torch.cuda.synchronize(dev)
    ok = True
    for slot in range(pool):
        outs[slot].zero_()
        encode(slot, B)
        dec(slot, slot % len(sets))
        torch.cuda.synchronize(dev)
        ok = ok and bool(torch.equal(outs[slot], segs[slot]))
    per = [e[0].elapsed_time(e[1]) * 1e-3 for e, _ in ev]
    t = sum(per) / len(per)
    by_set = {}
    for (e, i), x in zip(ev, per):
        by_set.setdefault(i, []).append(x * 1e6 / B)
    body = "straight-line" if L.ec_last_body(ctx) == _native.EC_BODY_STRAIGHT_LINE else "jump-table"
    return {"kernel": f"rs_matmul_dma<NW, 1> ({body} body, LDS-DMA staging)", "avg_us": round(t * 1e6, 2),
            "achieved_GBps": round(2 * S_PAD * B / t / 1e9, 1),
            "frac": round(2 * S_PAD * B / t / 1e9 / HBM_PEAK_GBPS, 4),
            "us_per_segment_by_set": {f"set{i}:m={K - sum(1 for x in sets[i] if x < K)}": round(sum(v) / len(v), 2)
                                      for i, v in sorted(by_set.items())},
            "verified": ok, "note": "informational, not in value (uplink's downloads do not reuse sets)"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # BENCH_DIST_BACKEND=gloo rehearses the N > 1 path on a one-GPU box (ranks share the
    # device, host-side collectives); the driver's multi-GPU runs use the default, RCCL.
    backend = os.environ.get("BENCH_DIST_BACKEND", "nccl")
    coll_dev = torch.device("cpu") if backend == "gloo" else None
    # BENCH_FORCE_DIST=1 (under torch.distributed.run) makes the process group and runs the bench's
    # collectives even at world size 1, so a one-GPU box exercises the RCCL path the 8-GPU run takes
    use_dist = world > 1 or os.environ.get("BENCH_FORCE_DIST") == "1"
    if use_dist:
        import torch.distributed as dist
        torch.cuda.set_device(local if backend != "gloo" else local % torch.cuda.device_count())
        if backend == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    L = _native.load(args.lib, partial=True) if args.lib else _native.load()
    if L.ec_set_device(torch.cuda.current_device()) != 0:
        raise RuntimeError("ec_set_device failed")
    ctx = ctypes.c_void_p()
    rc = L.ec_create(K, N, ESS, ctypes.byref(ctx))
    if rc != 0:
        raise RuntimeError(f"ec_create failed: {_native.strerror(rc)}")
    body = {"auto": _native.EC_BODY_AUTO, "jump-table": _native.EC_BODY_JUMP_TABLE,
            "straight-line": _native.EC_BODY_STRAIGHT_LINE}[args.body]
    if L.ec_set_body(ctx, body) != 0:
        raise RuntimeError("ec_set_body failed")

    # this rank's shard of configs[3] and the launches it takes
    first, count = shard_range(args.total_segments, world, rank)
    B = args.batch
    launches = [min(B, count - i) for i in range(0, count, B)]
    pool = 2  # slots of B distinct segments, cycled over the shard
    segs = [padded_segments(B, segment_seed(first + i * B), dev) for i in range(pool)]
    pieces = [torch.empty((B, N, PIECE), dtype=torch.uint8, device=dev) for _ in range(pool)]
    outs = [torch.empty((B, S_PAD), dtype=torch.uint8, device=dev) for _ in range(pool)]
    stream = torch.cuda.current_stream(dev)
    sptr = stream.cuda_stream

    def encode(slot, nb):
        r = L.ec_encode_segments(ctx, segs[slot].data_ptr(), nb, NSTRIPES, pieces[slot].data_ptr(), 0, sptr)
        if r:
            raise RuntimeError(_native.strerror(r))

    # the timed decode: a share set per segment, fresh every launch (ec_rebuild_segments_sets)
    def set_args(slot, sets_):
        """one call's arrays, made before the timed region (a Go caller holds its slices)"""
        n = len(sets_)
        flat = [x for st in sets_ for x in st]
        return (n, (ctypes.c_int * n)(*[K] * n), (ctypes.c_int * len(flat))(*flat),
                (ctypes.c_void_p * len(flat))(*[pieces[slot][g].data_ptr() + x * PIECE
                                                for g, st in enumerate(sets_) for x in st]),
                (ctypes.c_void_p * n)(*[outs[slot][g].data_ptr() for g in range(n)]), sets_)

    def decode(slot, a):
        n, nsh, nums, ptrs, optr, _ = a
        r = L.ec_rebuild_segments_sets(ctx, n, nsh, nums, ptrs, NSTRIPES, optr, sptr)
        if r:
            raise RuntimeError(_native.strerror(r))

    seed_base = 0x5E750000 + 1_000_003 * rank
    launch_no = [0]

    def fresh_args(slot, nb, all_parity_first=False):
        a = set_args(slot, fresh_launch_sets(seed_base + launch_no[0], nb, all_parity_first))
        launch_no[0] += 1
        return a

    def step_args():  # (every step's first segment is rebuilt from {51..79})
        return [fresh_args(b % pool, nb, b == 0) for b, nb in enumerate(launches)]

    def barrier():
        torch.cuda.synchronize(dev)
        if use_dist:
            import torch.distributed as dist
            dist.barrier()
        torch.cuda.synchronize(dev)

    def step(sargs, events=None):
        for b, nb in enumerate(launches):
            slot = b % pool
            if events is not None:
                # one marker per launch boundary: a launch pair starts at the previous pair's end
                # marker (a marker costs the stream ~4 us), only the first is extra
                if not events:
                    first = torch.cuda.Event(enable_timing=True)
                    first.record(stream)
                else:
                    first = events[-1][0][2]
                e = (first, torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                encode(slot, nb)
                e[1].record(stream)
                decode(slot, sargs[b])
                e[2].record(stream)
                events.append((e, nb, sargs[b][5]))
            else:
                encode(slot, nb)
                decode(slot, sargs[b])

    # every call's share sets and arrays, made before anything is timed (fresh per launch)
    warm_args = [step_args() for _ in range(args.warmup)]
    timed_args = [step_args() for _ in range(args.steps)]
    cycle = [[fresh_args(slot, B) for _ in range(8)] for slot in range(pool)]
    # warm-up: the clock settle (kernels loaded, share-set slots allocated), then W steps
    t_settle = time.perf_counter()
    i = 0
    while time.perf_counter() - t_settle < args.settle_s or i < 2 * pool:
        slot = i % pool
        encode(slot, B)
        decode(slot, cycle[slot][(i // pool) % 8])
        i += 1
        if i % (2 * pool) == 0:
            torch.cuda.synchronize(dev)
    for w in range(args.warmup):
        step(warm_args[w])
    barrier()

    # timed: exactly K steps; per-launch HIP events on the launch stream (torch's current stream)
    events = []
    t0 = time.perf_counter()
    for st_ in range(args.steps):
        step(timed_args[st_], events)
    barrier()
    wall = time.perf_counter() - t0

    seg_launched = sum(nb for _, nb, _ in events)
    t_enc = sum(e[0].elapsed_time(e[1]) for e, _, _ in events) * 1e-3  # s, all launches
    t_dec = sum(e[1].elapsed_time(e[2]) for e, _, _ in events) * 1e-3
    full = [(e, st_) for e, nb, st_ in events if nb == B]
    t_enc_full = sum(e[0].elapsed_time(e[1]) for e, _ in full) / max(len(full), 1) * 1e-3  # s per B-launch
    t_dec_full = sum(e[1].elapsed_time(e[2]) for e, _ in full) / max(len(full), 1) * 1e-3
    rows_timed = sorted(sum(1 for x in st if x >= K) for _, sets_ in full for st in sets_)
    # every rank's wall time (shard imbalance shows here) and a count of the ranks that took part
    rank_walls, ranks_seen = [round(wall, 6)], 1
    if use_dist:
        import torch.distributed as dist
        walls = [torch.zeros(1, dtype=torch.float64, device=coll_dev or dev) for _ in range(world)]
        dist.all_gather(walls, torch.tensor([wall], dtype=torch.float64, device=coll_dev or dev))
        rank_walls = [round(float(w.item()), 6) for w in walls]
        seen = torch.ones(1, dtype=torch.int64, device=coll_dev or dev)
        dist.all_reduce(seen, op=dist.ReduceOp.SUM)
        ranks_seen = int(seen.item())
        wall = max(rank_walls)

    # correctness (outside the timed region): every pool slot's segments encoded and rebuilt from
    # fresh share sets (one segment all parity) equal their input, and one segment's pieces match
    # the oracle
    verified = True
    for slot in range(pool):
        outs[slot].zero_()
        encode(slot, B)
        decode(slot, fresh_args(slot, B, True))
        torch.cuda.synchronize(dev)
        verified = verified and bool(torch.equal(outs[slot], segs[slot]))
    verified = verified and oracle_spot_check(pieces[0][0], segs[0][0])

    # informational, outside the timed region: the same decode from ONE warm share set per launch
    # (ec_rebuild_segments_batched, the set's straight-line code made and waited for before
    # timing) -- what a caller reusing a set gets; uplink's downloads do not (the timed leg)
    warm = warm_shared_set_leg(L, ctx, encode, pieces, outs, segs, pool, B, dev, stream, sptr)

    # informational, outside the timed region: the parity-only encode (data pieces are the
    # segment's own shares, served in place; the upload path of §8f row 1 uses this form), and
    # the encoder's own schedule without arithmetic (ec_encode_shape_probe, both forms).  Timed
    # like the headline encode -- each launch followed by a decode launch, per-launch events --
    # and also back to back, where a denser VALU body runs at a lower sustained clock.
    par = torch.empty((B, N - K, PIECE), dtype=torch.uint8, device=dev)

    def par_encode():
        if L.ec_encode_segments(ctx, segs[0].data_ptr(), B, NSTRIPES, par.data_ptr(), _native.EC_FLAG_PARITY_ONLY,
                                sptr):
            raise RuntimeError("parity-only encode failed")

    def shape_full():  # (writes pieces[0] with copies, not parity: re-encoded after)
        if L.ec_encode_shape_probe(ctx, segs[0].data_ptr(), B, NSTRIPES, pieces[0].data_ptr(), 0, sptr):
            raise RuntimeError("ec_encode_shape_probe failed")

    def shape_par():
        if L.ec_encode_shape_probe(ctx, segs[0].data_ptr(), B, NSTRIPES, par.data_ptr(), _native.EC_FLAG_PARITY_ONLY,
                                   sptr):
            raise RuntimeError("ec_encode_shape_probe (parity only) failed")

    def timed_like_headline(launch, reps=20):
        """(alternating with a decode launch, as timed; back to back) seconds per launch"""
        # the GPU idled through the checks above (oracle on the host): settle its clock again first,
        # as before the timed steps, so the launches are timed in the same steady state
        t_settle = time.perf_counter()
        j = 0
        while time.perf_counter() - t_settle < max(args.settle_s, 0.1):
            launch()
            decode(1 % pool, cycle[1 % pool][j % 8])
            j += 1
            torch.cuda.synchronize(dev)
        pev = []
        for r in range(reps):
            e = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            e[0].record(stream)
            launch()
            e[1].record(stream)
            decode(1 % pool, cycle[1 % pool][r % 8])
            pev.append(e)
        pe = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        pe[0].record(stream)
        for _ in range(reps):
            launch()
        pe[1].record(stream)
        pe[1].synchronize()
        return (sum(a.elapsed_time(b) for a, b in pev) / reps * 1e-3, pe[0].elapsed_time(pe[1]) / reps * 1e-3)

    t_par, t_par_b2b = timed_like_headline(par_encode)
    encode(0, B)
    torch.cuda.synchronize(dev)
    verified = verified and bool(torch.equal(par, pieces[0][:, K:]))
    shape_ok = hasattr(L, "ec_encode_shape_probe")
    t_shape = t_shape_b2b = t_shape_par = t_shape_par_b2b = None
    if shape_ok:
        t_shape, t_shape_b2b = timed_like_headline(shape_full)
        t_shape_par, t_shape_par_b2b = timed_like_headline(shape_par)
        encode(0, B)  # (pieces[0] holds the probe's copies: the real pieces again)
        torch.cuda.synchronize(dev)
    del par
    if use_dist:
        import torch.distributed as dist
        v = torch.tensor([1 if verified else 0], device=coll_dev or dev)
        dist.all_reduce(v, op=dist.ReduceOp.MIN)
        verified = bool(v.item())

    total_payload = args.steps * args.total_segments * S_PAD
    value = total_payload / 2**30 / wall
    enc_bytes = B * S_PAD * (1 + N / K)  # algorithmic bytes per encode launch of B segments
    dec_bytes = B * S_PAD * 2  # per decode launch
    enc_gbps = enc_bytes / t_enc_full / 1e9
    dec_gbps = dec_bytes / t_dec_full / 1e9
    enc_name = L.ec_encode_kernel_name(ctx).decode()
    kernels = {
        "encode": {"kernel": (f"{ENC_FULL_KERNEL} (special)" if enc_name == "special"
                              else f"rs_matmul_dma<7, 1> ({enc_name})"), "avg_us": round(t_enc_full * 1e6, 2),
                   "bytes_per_launch": int(enc_bytes), "achieved_GBps": round(enc_gbps, 1)},
        "decode": {"kernel": "rs_sets_prep + rs_matmul_sets<NW> (a share set per segment, decode rows solved on "
                             "the GPU, jump-table body, LDS-DMA staging)",
                   "avg_us": round(t_dec_full * 1e6, 2),
                   "bytes_per_launch": int(dec_bytes), "achieved_GBps": round(dec_gbps, 1),
                   "rows_per_segment": (f"{rows_timed[0]}..{rows_timed[-1]} (median {rows_timed[len(rows_timed) // 2]})"
                                        if rows_timed else None)},
        "decode_warm_shared_set": warm,
    }
    par_bytes = B * S_PAD * (1 + (N - K) / K)
    par_frac = round(par_bytes / t_par / 1e9 / HBM_PEAK_GBPS, 4)
    kernels["encode_parity_only"] = {
        "kernel": (ENC_PARITY_KERNEL if enc_name == "special" else "rs_matmul_dma<7, 1>")
                  + " (EC_FLAG_PARITY_ONLY)", "avg_us": round(t_par * 1e6, 2),
        "avg_us_back_to_back": round(t_par_b2b * 1e6, 2),
        "bytes_per_launch": int(par_bytes), "achieved_GBps": round(par_bytes / t_par / 1e9, 1),
        "frac": par_frac, "note": "informational, not in value"}
    shape_gbps = enc_bytes / t_shape / 1e9 if t_shape else None
    shape_par_gbps = par_bytes / t_shape_par / 1e9 if t_shape_par else None
    if shape_ok:
        kernels["encode_shape_probe"] = {
            "kernel": "rs_encode_shape<29, 80, 8, 4, true/false> (ec_encode_shape_probe: the encoder's body "
                      "without its multiply-accumulate)",
            "full_avg_us": round(t_shape * 1e6, 2), "full_avg_us_back_to_back": round(t_shape_b2b * 1e6, 2),
            "full_GBps": round(shape_gbps, 1),
            "parity_only_avg_us": round(t_shape_par * 1e6, 2),
            "parity_only_avg_us_back_to_back": round(t_shape_par_b2b * 1e6, 2),
            "parity_only_GBps": round(shape_par_gbps, 1),
            "note": "same loaders, LDS ring, tile queue, slicing and stores as the encoder, no GF arithmetic; "
                    "timed like the headline encode (each launch followed by a decode launch) and back to back"}
    # SURVEY §8d, VERDICT r4 item 4: on-box ceilings next to the spec peak -- the library's own
    # streaming kernels (ec_bw_probe, no arithmetic) in the read:write mixes of the kernels measured
    # here, in the best shapes of the round-2 probes; outside the timed region
    ceil = on_box_ceilings(L, dev, stream) if hasattr(L, "ec_bw_probe") else {}
    dominant = "encode" if t_enc_full >= t_dec_full else "decode"
    dk = kernels[dominant]
    # PMC traffic of the dominant kernel, from the record tools/prof_round.sh wrote for one build:
    # used only when that build is the library running here (ec_build_id) and the batch matches
    traffic, traffic_note = None, None
    try:
        with open(args.traffic_json) as fh:
            tj = json.load(fh)
        build = L.ec_build_id().decode()
        if tj.get("build_id") != build:
            traffic_note = f"{args.traffic_json} was taken from build {tj.get('build_id')}, this is {build}"
        elif tj.get("segments_per_launch") != B:
            traffic_note = f"{args.traffic_json} is per launch of {tj.get('segments_per_launch')} segments, not {B}"
        else:
            traffic = tj.get(dominant, {}).get("hbm_bytes_per_launch")
            traffic_note = f"rocprofv3 FETCH_SIZE/WRITE_SIZE of build {build}: {tj.get(dominant, {}).get('kernels')}"
    except (OSError, ValueError) as e:
        traffic_note = f"no PMC record: {e}"
    line = {
        "metric": "GiB/s erasure encode+decode (device-resident), RS(29,80) 64 MiB segments",
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(wall / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "u8",
        "data": f"synthetic (device-generated random segments, PadReader-padded; pool of 2 x {B} per rank, cycled)",
        "config": {"workload": "RS(29,80) encode+decode of a batch of 64 MiB segments sharded over the GPUs "
                               "(BASELINE configs[3], each segment as configs[1]+[2])",
                   "k": K, "n": N, "erasure_share_size": ESS, "total_segments_per_step": args.total_segments,
                   "segments_this_rank": count, "segments_per_launch": B, "stripes_per_segment": NSTRIPES,
                   "decode_share_sets": "a fresh seeded 29-subset per segment and launch (each step's first "
                                        "segment from {51..79}); no plan made or warmed",
                   "parallelism": f"segments sharded over {world} GPU(s), no collective"},
        "roofline": {"bound": "hbm", "kernel": dominant, "achieved": round(dk["achieved_GBps"], 1),
                     "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": round(dk["achieved_GBps"] / HBM_PEAK_GBPS, 4),
                     "traffic": traffic, "traffic_note": traffic_note, "frac_parity_only_encode": par_frac,
                     "frac_decode": round(dec_gbps / HBM_PEAK_GBPS, 4),
                     "copy_GBps_on_box": _r(ceil.get("copy"), 1),
                     "encode_mix_GBps_on_box": _r(ceil.get("encode_mix"), 1),
                     "parity_mix_GBps_on_box": _r(ceil.get("parity_mix"), 1),
                     "frac_of_mix": _ratio(enc_gbps, ceil.get("encode_mix")),
                     "frac_of_mix_parity_only": _ratio(par_bytes / t_par / 1e9, ceil.get("parity_mix")),
                     "frac_decode_of_copy": _ratio(dec_gbps, ceil.get("copy")),
                     "encode_shape_GBps_on_box": _r(shape_gbps, 1),
                     "parity_shape_GBps_on_box": _r(shape_par_gbps, 1),
                     "frac_of_shape": _ratio(enc_gbps, shape_gbps),
                     "frac_of_shape_parity_only": _ratio(par_bytes / t_par / 1e9, shape_par_gbps),
                     "shape_frac_of_peak": _ratio(shape_gbps, HBM_PEAK_GBPS),
                     "ceilings_note": "ec_bw_probe: one-shot grid, each wave R KiB in / W KiB out, 16 B per lane, "
                                      "non-temporal, no arithmetic; copy 1:1, encode mix 4:11 (the encode's 29:80), "
                                      "parity mix 4:7 (29:51); 1 GiB read, median of 10 launches; encode shape: "
                                      "the encoder's own schedule without arithmetic (ec_encode_shape_probe), timed "
                                      "as the encode is"},
        "kernels": kernels,
        "encode_gibps": round(B * S_PAD / 2**30 / t_enc_full, 2),
        "decode_gibps": round(B * S_PAD / 2**30 / t_dec_full, 2),
        "gpu_busy_s": round(t_enc + t_dec, 4),
        "segments_timed_this_rank": seg_launched,
        "ranks_seen": ranks_seen,
        "collectives": backend if use_dist else None,
        "rank_wall_s": rank_walls,
        "build_id": L.ec_build_id().decode(),
        "verified": verified,
    }
    # after the timed region, on rank 0 at every world size: the decode with a
    # fresh share set per segment, the reference benchmark's other configurations, the CPU baseline
    if rank == 0 and hasattr(L, "ec_rebuild_segments_sets"):  # (an older --lib build lacks it)
        line["fresh_share_sets"] = fresh_sets_leg(L, ctx, dev, sptr)
    if rank == 0 and not args.no_other_configs:
        line["other_configs"] = other_configs(L, dev, sptr)
        for key, val in line.get("fresh_share_sets", {}).items():  # (VERDICT r4 item 1 asks for them here too)
            if key != "note":
                line["other_configs"][f"RS(29,80) rebuild, {key}"] = val
        line["other_configs"]["RS(29,80) rebuild, a new share set every launch"] = fresh_share_sets(L, dev, sptr)
        if hasattr(L, "ec_decode_segments_batched"):
            line["other_configs"]["RS(29,80) decode with error detection"] = decode_with_detection(L, dev, sptr)
    if rank == 0 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(args.cpu_sample_s)
    if use_dist:  # the other ranks wait for rank 0's informational legs
        import torch.distributed as dist
        dist.barrier()
    if rank == 0:
        print(json.dumps(line), flush=True)
    L.ec_destroy(ctx)
    if use_dist:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
