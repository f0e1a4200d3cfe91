#!/usr/bin/env python3
"""Developer measurement: the upload side end to end from host memory --
a 64 MiB segment in a pinned buffer.Backend to all RS(29,80) pieces in host
memory through SegmentPieceReader (PadReader + one streamed parity-only
engine call, ec_upload_begin; data pieces served from the padded segment).
PCIe-inclusive; never the bench.py value.

Reports, median of 10 after 2 untimed:
  * first byte: from the reader's first piece_reader() call to the first
    4 KiB of a parity piece in hand (what an upload waits before it can send);
  * whole segment: until every parity piece is in host memory;
  * the same segment through the blocking ec_encode_segments_host call
    (the round-3 path: no reader returns before the whole segment is done)."""
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from uplink_amd import _native as NAT  # noqa: E402
from uplink_amd import eestream, segment  # noqa: E402

K, N, ESS, SEG = 29, 80, 256, 64 * 1024 * 1024


def main():
    chunk = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    rs = eestream.RedundancyStrategy(eestream.RSScheme(eestream.new_fec(K, N), ESS), 0, 0)
    be = segment.PinnedBackend()
    be.write(np.random.default_rng(1).integers(0, 256, SEG, dtype=np.uint8))
    stripe = K * ESS
    stripes = (SEG + 4 + stripe - 1) // stripe
    parity_bytes = (N - K) * stripes * ESS
    first, whole, blocking = [], [], []
    lib = NAT.load()
    for it in range(12):
        spr = segment.SegmentPieceReader(be, rs, chunk_stripes=chunk)
        t0 = time.perf_counter()
        b = spr.piece_reader(K).read(4096)
        t1 = time.perf_counter()
        spr._wait(stripes * ESS)
        t2 = time.perf_counter()
        assert len(b) == 4096
        spr.close()
        # the blocking path on the same (already padded) segment
        out = segment.pinned_pool.get(parity_bytes)
        t3 = time.perf_counter()
        rc = lib.ec_encode_segments_host(rs.scheme.ctx, be._mem.ptr, 1, stripes, out.ptr, NAT.EC_FLAG_PARITY_ONLY)
        t4 = time.perf_counter()
        assert rc == 0
        segment.pinned_pool.put(out)
        if it >= 2:
            first.append(t1 - t0)
            whole.append(t2 - t0)
            blocking.append(t4 - t3)
    f, w, bl = (float(np.median(x)) for x in (first, whole, blocking))
    print(f"streamed upload (chunk {'library default' if not chunk else chunk}): first parity byte after "
          f"{f * 1e3:.3f} ms ({100 * f / w:.1f} % of the segment), whole segment {w * 1e3:.2f} ms = "
          f"{SEG / w / 2**30:.2f} GiB/s payload, {(SEG + parity_bytes) / w / 1e9:.1f} GB/s PCIe")
    print(f"blocking ec_encode_segments_host (parity only): {bl * 1e3:.2f} ms = {SEG / bl / 2**30:.2f} GiB/s payload; "
          f"streamed / blocking whole-segment time {w / bl:.3f}")
    be.close()


if __name__ == "__main__":
    main()
