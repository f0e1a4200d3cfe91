"""Developer experiment: time the RS(29,80) encode (full and parity-only,
16 x 64 MiB segments per launch, as bench.py) in library variants built by
tools/exp/build_enc_variants.sh, interleaved A/B/A/B so box drift cancels, and
check every variant's pieces against the product library's.
  python tools/exp/enc_variants.py tools/exp/bin/var_*/libuplink_ec.so
"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench as B  # noqa: E402
from uplink_amd import _native  # noqa: E402


def load(path):
    lib = ctypes.CDLL(path)
    for name, (res, args) in _native.SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


def main(paths):
    dev = torch.device("cuda", 0)
    nb = 16
    segs = B.padded_segments(nb, 0, dev)
    pieces = torch.empty((nb, B.N, B.PIECE), dtype=torch.uint8, device=dev)
    ref = None
    s = torch.cuda.current_stream().cuda_stream
    libs = []
    for p in [_native.LIB_PATH] + paths:
        L = load(p)
        ctx = ctypes.c_void_p()
        assert L.ec_create(B.K, B.N, B.ESS, ctypes.byref(ctx)) == 0
        pieces.zero_()
        assert L.ec_encode_segments(ctx, segs.data_ptr(), nb, B.NSTRIPES, pieces.data_ptr(), 0, s) == 0
        torch.cuda.synchronize()
        if ref is None:
            ref = pieces.clone()
            ok = True
        else:
            ok = bool(torch.equal(pieces, ref))
        tag = os.path.basename(os.path.dirname(p)) if p != _native.LIB_PATH else "product"
        print(f"{tag:28s} kernel={L.ec_encode_kernel_name(ctx).decode()!r} pieces_equal={ok}", flush=True)
        libs.append((tag, L, ctx))

    def t(L, ctx, flags, it=20):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        for _ in range(3):
            L.ec_encode_segments(ctx, segs.data_ptr(), nb, B.NSTRIPES, pieces.data_ptr(), flags, s)
        e0.record()
        for _ in range(it):
            L.ec_encode_segments(ctx, segs.data_ptr(), nb, B.NSTRIPES, pieces.data_ptr(), flags, s)
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / it / nb

    res = {tag: {"full": [], "parity": []} for tag, _, _ in libs}
    for rnd in range(3):
        for tag, L, ctx in libs:
            res[tag]["full"].append(t(L, ctx, 0))
            res[tag]["parity"].append(t(L, ctx, _native.EC_FLAG_PARITY_ONLY))
    full_bytes = B.S_PAD * (1 + B.N / B.K)
    par_bytes = B.S_PAD * (1 + (B.N - B.K) / B.K)
    for tag, r in res.items():
        f = min(r["full"])
        pa = min(r["parity"])
        print(f"{tag:28s} full {f:6.2f} us/seg ({full_bytes / f / 1e6:5.3f} TB/s)  "
              f"parity {pa:6.2f} us/seg ({par_bytes / pa / 1e6:5.3f} TB/s)   all: "
              f"{' '.join(f'{x:.1f}' for x in r['full'])} | {' '.join(f'{x:.1f}' for x in r['parity'])}", flush=True)


if __name__ == "__main__":
    main(sys.argv[1:])
