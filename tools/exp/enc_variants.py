"""Developer experiment: time the compile-time encoder (full and parity-only,
16 x 64 MiB segments per launch, as bench.py) for RS(29,80) and the reference
benchmark's library-built configurations in library variants built by
tools/exp/build_enc_variants.sh, interleaved A/B/A/B so box drift cancels,
and check every variant's pieces against the product library's.
  python tools/exp/enc_variants.py tools/exp/bin/var_*/libuplink_ec.so
"""
import ctypes
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from uplink_amd import _native  # noqa: E402

CONFIGS = [(29, 80), (20, 50), (30, 60), (50, 80), (20, 60)]
if os.environ.get("ENC_ONLY"):  # e.g. ENC_ONLY=50,80
    CONFIGS = [tuple(int(x) for x in os.environ["ENC_ONLY"].split(","))]
COOL_S = float(os.environ.get("ENC_COOL_S", "0"))  # idle time before each timed loop
ESS = 256
RAW = 64 << 20


def load(path):
    lib = ctypes.CDLL(path)
    for name, (res, args) in _native.SIGNATURES.items():
        if not hasattr(lib, name):  # an older build for the A/B
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


def main(paths):
    dev = torch.device("cuda", 0)
    nb = 16
    s = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    bufs = {}
    for k, n in CONFIGS:
        stripes = (RAW + 4 + k * ESS - 1) // (k * ESS)
        segs = torch.randint(0, 256, (nb, stripes * k * ESS), dtype=torch.uint8, device=dev, generator=g)
        bufs[(k, n)] = (stripes, segs, torch.empty((nb, n, stripes * ESS), dtype=torch.uint8, device=dev))
    libs = []
    refs = {}
    for p in [_native.LIB_PATH] + paths:
        L = load(p)
        tag = os.path.basename(os.path.dirname(p)) if p != _native.LIB_PATH else "product"
        ctxs = {}
        for (k, n), (stripes, segs, pieces) in bufs.items():
            ctx = ctypes.c_void_p()
            assert L.ec_create(k, n, ESS, ctypes.byref(ctx)) == 0
            ctxs[(k, n)] = ctx
            pieces.zero_()
            assert L.ec_encode_segments(ctx, segs.data_ptr(), nb, stripes, pieces.data_ptr(), 0, s) == 0
            torch.cuda.synchronize()
            if (k, n) not in refs:
                refs[(k, n)] = pieces.clone()
            elif not torch.equal(pieces, refs[(k, n)]):
                # timing-only variants (experiment switches that drop the math or the traffic) differ on purpose
                print(f"{tag:20s} pieces DIFFER from the product's for RS{(k, n)} (timing only)", flush=True)
        print(f"{tag:20s} checked against the product's pieces for {CONFIGS}", flush=True)
        libs.append((tag, L, ctxs))

    def t(L, ctx, kn, flags, it=20):
        stripes, segs, pieces = bufs[kn]
        if COOL_S:
            time.sleep(COOL_S)
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        for _ in range(3):
            L.ec_encode_segments(ctx, segs.data_ptr(), nb, stripes, pieces.data_ptr(), flags, s)
        e0.record()
        for _ in range(it):
            L.ec_encode_segments(ctx, segs.data_ptr(), nb, stripes, pieces.data_ptr(), flags, s)
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / it / nb

    res = {(tag, kn, f): [] for tag, _, _ in libs for kn in CONFIGS for f in (0, 1)}
    for rnd in range(3):
        for tag, L, ctxs in libs:
            for kn in CONFIGS:
                # ENC_PO_FIRST=1 times the parity-only launch before the full one (the launch
                # timed second runs on a chip heated by the first)
                for f in ((1, 0) if os.environ.get("ENC_PO_FIRST") == "1" else (0, 1)):
                    res[(tag, kn, f)].append(t(L, ctxs[kn], kn, _native.EC_FLAG_PARITY_ONLY if f else 0))
    print("us per segment (min of 3 rounds), TB/s algorithmic; full | parity-only")
    for kn in CONFIGS:
        k, n = kn
        stripes = bufs[kn][0]
        sp = stripes * k * ESS
        for tag, _, _ in libs:
            f, pa = min(res[(tag, kn, 0)]), min(res[(tag, kn, 1)])
            print(f"RS{kn!s:9s} {tag:20s} full {f:6.2f} ({sp * (1 + n / k) / f / 1e6:5.3f})  "
                  f"parity {pa:6.2f} ({sp * (1 + (n - k) / k) / pa / 1e6:5.3f})", flush=True)


if __name__ == "__main__":
    main(sys.argv[1:])
