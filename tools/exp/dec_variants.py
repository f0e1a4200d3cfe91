"""Developer experiment: time the RS(29,80) rebuild (16 x 64 MiB segments per
launch, bench.py's layout) for share sets with m = 0 .. 29 missing data
shares in library variants (tools/exp/build_enc_variants.sh), interleaved
so box drift cancels; every
rebuild is checked against the segments it came from.
  python tools/exp/dec_variants.py tools/exp/bin/var_*/libuplink_ec.so
"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench as B  # noqa: E402
from enc_variants import load  # noqa: E402
from uplink_amd import _native  # noqa: E402


def main(paths):
    dev = torch.device("cuda", 0)
    nb = 16
    segs = B.padded_segments(nb, 0, dev)
    pieces = torch.empty((nb, B.N, B.PIECE), dtype=torch.uint8, device=dev)
    out = torch.empty((nb, B.S_PAD), dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    rng = np.random.default_rng(5)
    sets = {}
    for m in (0, 8, 16, 19, 22, 29):
        data = sorted(rng.choice(B.K, B.K - m, replace=False).tolist())
        par = sorted((B.K + rng.choice(B.N - B.K, m, replace=False)).tolist())
        sets[m] = data + par
    libs = []
    for p in [_native.LIB_PATH] + paths:
        L = load(p)
        ctx = ctypes.c_void_p()
        assert L.ec_create(B.K, B.N, B.ESS, ctypes.byref(ctx)) == 0
        tag = os.path.basename(os.path.dirname(p)) if p != _native.LIB_PATH else "product"
        libs.append((tag, L, ctx))
    L0, c0 = libs[0][1], libs[0][2]
    assert L0.ec_encode_segments(c0, segs.data_ptr(), nb, B.NSTRIPES, pieces.data_ptr(), 0, s) == 0
    base = pieces.data_ptr()

    def rebuild(L, ctx, m):
        nums = (ctypes.c_int * B.K)(*sets[m])
        ptrs = (ctypes.c_void_p * B.K)(*[base + j * B.PIECE for j in sets[m]])
        return L.ec_rebuild_segments_batched(ctx, B.K, nums, ptrs, B.NSTRIPES, nb, B.N * B.PIECE, B.S_PAD,
                                            out.data_ptr(), s)

    for tag, L, ctx in libs:
        ok = True
        for m in sets:
            out.zero_()
            assert rebuild(L, ctx, m) == 0
            torch.cuda.synchronize()
            ok = ok and bool(torch.equal(out, segs))
        print(f"{tag:20s} rebuild_equal={ok}", flush=True)

    def t(L, ctx, m, it=20):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        for _ in range(3):
            rebuild(L, ctx, m)
        e0.record()
        for _ in range(it):
            rebuild(L, ctx, m)
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / it / nb

    res = {tag: {m: [] for m in sets} for tag, _, _ in libs}
    for rnd in range(3):
        for tag, L, ctx in libs:
            for m in sets:
                res[tag][m].append(t(L, ctx, m))
    print("us per segment (min of 3 rounds); TB/s at 2 x S_PAD per segment")
    print(f"{'':20s} " + " ".join(f"{'m=' + str(m):>14s}" for m in sets))
    for tag, r in res.items():
        print(f"{tag:20s} " + " ".join(f"{min(v):6.2f} ({2 * B.S_PAD / min(v) / 1e6:4.2f})" for v in r.values()),
              flush=True)


if __name__ == "__main__":
    main(sys.argv[1:])
