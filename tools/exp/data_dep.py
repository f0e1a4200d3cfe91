"""Developer experiment: does the data itself change the kernels' speed?
Times the product RS(29,80) encode (full and parity-only) and the rebuild
(m = 0 and m = 29) of 16 x 64 MiB segments holding random bytes, a constant
byte, and zeros, interleaved over 3 rounds (min per case).  The round-3 shape
probes ran on memset buffers; the product and bench.py run on random data.
  python tools/exp/data_dep.py
"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench as B  # noqa: E402
from uplink_amd import _native  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    nb = 16
    L = _native.load()
    ctx = ctypes.c_void_p()
    assert L.ec_create(B.K, B.N, B.ESS, ctypes.byref(ctx)) == 0
    s = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    kinds = {
        "random": torch.randint(0, 256, (nb, B.S_PAD), dtype=torch.uint8, device=dev, generator=g),
        "const 0x5a": torch.full((nb, B.S_PAD), 0x5A, dtype=torch.uint8, device=dev),
        "zeros": torch.zeros((nb, B.S_PAD), dtype=torch.uint8, device=dev),
    }
    pieces = {kd: torch.empty((nb, B.N, B.PIECE), dtype=torch.uint8, device=dev) for kd in kinds}
    out = torch.empty((nb, B.S_PAD), dtype=torch.uint8, device=dev)
    for kd, segs in kinds.items():
        assert L.ec_encode_segments(ctx, segs.data_ptr(), nb, B.NSTRIPES, pieces[kd].data_ptr(), 0, s) == 0
    torch.cuda.synchronize()
    sets = {"m=0": list(range(B.K)), "m=29": list(range(B.N - B.K, B.N))}

    def enc(kd, flags):
        return L.ec_encode_segments(ctx, kinds[kd].data_ptr(), nb, B.NSTRIPES, pieces[kd].data_ptr(), flags, s)

    def reb(kd, m):
        nums = (ctypes.c_int * B.K)(*sets[m])
        base = pieces[kd].data_ptr()
        ptrs = (ctypes.c_void_p * B.K)(*[base + j * B.PIECE for j in sets[m]])
        return L.ec_rebuild_segments_batched(ctx, B.K, nums, ptrs, B.NSTRIPES, nb, B.N * B.PIECE, B.S_PAD,
                                            out.data_ptr(), s)

    cases = [("encode full", lambda kd: enc(kd, 0)), ("encode parity-only", lambda kd: enc(kd, _native.EC_FLAG_PARITY_ONLY)),
             ("rebuild m=0", lambda kd: reb(kd, "m=0")), ("rebuild m=29", lambda kd: reb(kd, "m=29"))]
    res = {}
    for _ in range(3):
        for name, f in cases:
            for kd in kinds:
                for _w in range(3):
                    assert f(kd) == 0
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record()
                for _i in range(20):
                    f(kd)
                e1.record()
                torch.cuda.synchronize()
                res.setdefault((name, kd), []).append(e0.elapsed_time(e1) * 1e3 / 20 / nb)
    print("us per 64 MiB segment (min of 3 rounds of 20 launches of 16 segments)")
    for name, _ in cases:
        print(f"{name:20s} " + "  ".join(f"{kd} {min(res[(name, kd)]):6.2f}" for kd in kinds), flush=True)


if __name__ == "__main__":
    main()
