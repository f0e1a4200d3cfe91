#!/usr/bin/env python3
"""Developer measurement: the upload side end to end from host memory --
a 64 MiB segment in a pinned buffer.Backend to all RS(29,80) pieces in host
memory through SegmentPieceReader (PadReader + one parity-only engine call;
data pieces served from the padded segment).  PCIe-inclusive; never the
bench.py value."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from uplink_amd import eestream, segment  # noqa: E402

K, N, ESS, SEG = 29, 80, 256, 64 * 1024 * 1024
rs = eestream.RedundancyStrategy(eestream.RSScheme(eestream.new_fec(K, N), ESS), 0, 0)
be = segment.PinnedBackend()
be.write(np.random.default_rng(1).integers(0, 256, SEG, dtype=np.uint8))
times = []
for it in range(12):
    spr = segment.SegmentPieceReader(be, rs)
    t0 = time.perf_counter()
    spr._prepare()
    times.append(time.perf_counter() - t0)
    spr.close()
t = float(np.median(times[2:]))
parity = (N - K) * (SEG + 4096) // K
print(f"segment -> all {N} pieces (parity over PCIe, data from the host segment): {t * 1e3:.2f} ms, "
      f"{SEG / t / 2**30:.2f} GiB/s payload, {(SEG + parity) / t / 1e9:.1f} GB/s PCIe")
