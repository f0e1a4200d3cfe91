"""Developer experiment (not product), round 4: does where the buffers sit in
HBM move the RS(29,80) encode and rebuild?

Round 3's shape probe (profiles/r03/enc/shape_probe2_v6_allocs_box2.log) ran
one kernel on three separately allocated buffer sets and saw 5.6 vs 6.5 TB/s
by allocation.  Here the product library's ec_encode_segments (16 segments
per launch, as bench.py) and ec_rebuild_segments_batched (all-parity set) run
on
  * placements inside ONE large allocation (same physical pages, different
    offsets and orders of the segment and piece blocks), and
  * separately allocated buffer pairs,
interleaved over rounds on one device, HIP-event time per launch.

  python tools/exp/placement_probe.py [--rounds 3] [--sep 4]
"""
from __future__ import annotations

import argparse
import ctypes
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from uplink_amd import _native  # noqa: E402

K, N, ESS = 29, 80, 256
NSTRIPES = (64 * 1024 * 1024 + 4 + K * ESS - 1) // (K * ESS)
S_PAD, PIECE = NSTRIPES * K * ESS, NSTRIPES * ESS
B = 16
SB, PB = B * S_PAD, B * N * PIECE
MiB = 1 << 20


def al(x, a=2 * MiB):
    return (x + a - 1) // a * a


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--sep", type=int, default=4, help="separately allocated buffer pairs")
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    L = _native.load()
    ctx = ctypes.c_void_p()
    assert L.ec_create(K, N, ESS, ctypes.byref(ctx)) == 0
    stream = torch.cuda.current_stream(dev)
    sptr = stream.cuda_stream
    src = torch.randint(0, 256, (SB,), dtype=torch.uint8, device=dev)

    arena_bytes = al(SB) + al(PB) + 64 * MiB
    arena = torch.empty(2 * arena_bytes, dtype=torch.uint8, device=dev)
    base = arena.data_ptr()
    placements = []  # (name, segs_ptr, pieces_ptr, holder)
    off_p = al(SB)
    placements.append(("arena: segs@0 pieces@2M-aligned end of segs", base, base + off_p, None))
    placements.append(("arena: pieces@0 segs@end of pieces", base + al(PB), base, None))
    for d in (2, 4, 6, 32):
        placements.append((f"arena: segs@0 pieces@+{d}MiB", base, base + off_p + d * MiB, None))
    placements.append(("arena: segs@+64KiB pieces@+0", base + 64 * 1024, base + off_p + 2 * MiB, None))
    placements.append(("arena: second half (segs, pieces)", base + arena_bytes, base + arena_bytes + off_p, None))
    for i in range(args.sep):
        s = torch.empty(SB, dtype=torch.uint8, device=dev)
        p = torch.empty(PB, dtype=torch.uint8, device=dev)
        placements.append((f"separate allocation pair {i}", s.data_ptr(), p.data_ptr(), (s, p)))
    print(f"arena base {base:#x}; separate: " +
          ", ".join(f"{pl[1]:#x}/{pl[2]:#x}" for pl in placements if pl[3] is not None), flush=True)

    def view(ptr):
        # the placement's segment block as a tensor (a slice of the arena or the separate buffer)
        for _, sp, _, h in placements:
            if sp == ptr and h is not None:
                return h[0]
        return arena[ptr - base: ptr - base + SB]

    back = torch.empty(SB, dtype=torch.uint8, device=dev)
    nums = (ctypes.c_int * K)(*range(N - K, N))

    def enc(sp, pp):
        assert L.ec_encode_segments(ctx, sp, B, NSTRIPES, pp, 0, sptr) == 0

    def dec(pp):
        ptrs = (ctypes.c_void_p * K)(*[pp + j * PIECE for j in range(N - K, N)])
        assert L.ec_rebuild_segments_batched(ctx, K, nums, ptrs, NSTRIPES, B, N * PIECE, S_PAD, back.data_ptr(),
                                             sptr) == 0

    for name, sp, pp, _ in placements:
        view(sp).copy_(src)
    torch.cuda.synchronize()
    # settle: 0.5 s of launches
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.5:
        enc(placements[0][1], placements[0][2])
        dec(placements[0][2])
        torch.cuda.synchronize()
    res = {name: ([], []) for name, *_ in placements}
    for r in range(args.rounds):
        for name, sp, pp, _ in placements:
            view(sp).copy_(src)  # placements overlap: refresh this one's segments
            for _ in range(2):
                enc(sp, pp)
                dec(pp)
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            ev[0].record(stream)
            for _ in range(args.reps):
                enc(sp, pp)
            ev[1].record(stream)
            for _ in range(args.reps):
                dec(pp)
            ev[2].record(stream)
            ev[2].synchronize()
            res[name][0].append(ev[0].elapsed_time(ev[1]) * 1e3 / args.reps)
            res[name][1].append(ev[1].elapsed_time(ev[2]) * 1e3 / args.reps)
            assert torch.equal(back, src), f"rebuild mismatch at {name}"
    eb, db = SB * (1 + N / K), 2 * SB
    print(f"{'placement':52s} {'encode us/launch (rounds)':>40s}  enc TB/s  {'rebuild us':>28s}  reb TB/s")
    for name, (e, d) in res.items():
        me, md = sorted(e)[len(e) // 2], sorted(d)[len(d) // 2]
        print(f"{name:52s} {' '.join(f'{x:7.1f}' for x in e):>40s}  {eb / me / 1e6:6.3f}  "
              f"{' '.join(f'{x:6.1f}' for x in d):>28s}  {db / md / 1e6:6.3f}", flush=True)
    L.ec_destroy(ctx)


if __name__ == "__main__":
    main()
