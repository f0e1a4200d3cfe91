#!/usr/bin/env python3
"""Developer measurement: ErasureScheme.Decode with error detection over a run
of stripes (ec_decode: the re-encode check of every column, then
Berlekamp-Welch on the flagged columns; stripe.go:407-408 with
forceErrorDetection, §8f row 3), host buffers, RS(29,80) with k+2 and k+4
shares of 1 MiB (4096 stripes of 256 B each): no errors, one corrupted share
(every column flagged) and sparse corruption."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from uplink_amd import eestream  # noqa: E402

K, N, LN = 29, 80, 1 << 20


def main():
    sch = eestream.RSScheme(eestream.new_fec(K, N), 256)
    rng = np.random.default_rng(4)
    data = rng.integers(0, 256, K * LN, dtype=np.uint8)  # LN / 256 stripes
    allp = sch.encode_stripes(data)  # [n][LN]: piece i over the run of stripes
    want = allp[:K].reshape(-1)      # Decode of whole-run shares = the k data pieces, concatenated
    res = {}
    for extra in (2, 4):
        nums = list(range(N - K - extra, N))
        base = [allp[i].copy() for i in nums]
        res[f"k+{extra}"] = {}
        for case in ("clean", "one share corrupted", "sparse (1 in 4096 columns)"):
            shares = [eestream.Share(nu, b.copy()) for nu, b in zip(nums, base)]
            if case == "one share corrupted":
                shares[3].data[:] ^= 0x5A
            elif case.startswith("sparse"):
                shares[1].data[::4096] ^= 0x11
            t0 = time.perf_counter()
            try:
                ok = bool(np.array_equal(sch.decode(None, shares), want))
            except eestream.InfectiousError:
                ok = False
            dt = time.perf_counter() - t0
            res[f"k+{extra}"][case] = {"ms": round(dt * 1e3, 2), "GiBps_payload": round(K * LN / dt / 2**30, 2),
                                      "decoded": ok}
    print(json.dumps({"metric": "ErasureScheme.Decode over a run of stripes (host buffers)", "share_bytes": LN,
                      "results": res}))


if __name__ == "__main__":
    main()
