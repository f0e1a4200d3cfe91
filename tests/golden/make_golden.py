"""Generate the golden fixtures under tests/golden/ from the oracle.

The reference (Go + storj.io/infectious) cannot run here (no Go toolchain, the
module is not vendored), so these vectors come from the CPU restatement in
oracle/ (pinned by the checks in tests/test_oracle.py: SURVEY Appendix A
fingerprints, zfec-vs-Lagrange agreement, round trips).  Inputs are seeded
(numpy default_rng(20261015)), per SURVEY.md §8c.

    python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import oracle as O  # noqa: E402

CASES = [  # (k, n, ess, stripes)
    (2, 4, 8, 1),
    (4, 10, 256, 4),
    (29, 80, 256, 2),
    (20, 60, 4096, 1),
    (3, 7, 1024, 3),
]


def main():
    rng = np.random.default_rng(20261015)
    manifest = {"seed": 20261015, "generator": "oracle/infectious_oracle.c (zfec construction)", "cases": []}
    for k, n, ess, stripes in CASES:
        seg = rng.integers(0, 256, stripes * k * ess, dtype=np.uint8)
        f = O.FEC(k, n)
        pieces = f.encode_segment(seg, ess)
        name = f"rs_{k}_{n}_ess{ess}_s{stripes}.npz"
        np.savez_compressed(os.path.join(HERE, name), segment=seg, pieces=pieces, generator=f.enc)
        manifest["cases"].append({
            "file": name, "k": k, "n": n, "ess": ess, "stripes": stripes,
            "generator_sha256": hashlib.sha256(f.enc.tobytes()).hexdigest(),
            "pieces_sha256": hashlib.sha256(pieces.tobytes()).hexdigest(),
            "segment_sha256": hashlib.sha256(seg.tobytes()).hexdigest(),
        })
    with open(os.path.join(HERE, "manifest.json"), "w") as fh:
        json.dump(manifest, fh, indent=1)


if __name__ == "__main__":
    main()
