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
    (the round-3 path: no reader returns before the whole segment is done);
  * all of it again with hash_pieces=True (EC_FLAG_HASH_PIECES: the BLAKE3 of
    every piece folded chunk by chunk as the segment streams), and the time
    until every piece hash is known."""
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
    lib = NAT.load()
    res = {}
    for hashed in (False, True):
        first, whole, hashes, blocking, begin = [], [], [], [], []
        for it in range(12):
            spr = segment.SegmentPieceReader(be, rs, chunk_stripes=chunk, hash_pieces=hashed)
            t0 = time.perf_counter()
            spr._prepare()  # pad + ec_upload_begin (everything queued)
            tb = time.perf_counter()
            r = spr.piece_reader(K)
            b = r.read(4096)
            t1 = time.perf_counter()
            spr._wait(stripes * ESS)
            t2 = time.perf_counter()
            if hashed:
                spr.piece_hash(N - 1)
            t3 = time.perf_counter()
            assert len(b) == 4096
            r.close()
            spr.close()
            # the blocking path on the same (already padded) segment
            out = segment.pinned_pool.get(parity_bytes)
            hb = np.zeros((N, 32), dtype=np.uint8)
            t4 = time.perf_counter()
            if hashed:
                rc = lib.ec_encode_segments_host_hashed(rs.scheme.ctx, be._mem.ptr, 1, stripes, out.ptr,
                                                        hb.ctypes.data, NAT.EC_FLAG_PARITY_ONLY)
            else:
                rc = lib.ec_encode_segments_host(rs.scheme.ctx, be._mem.ptr, 1, stripes, out.ptr,
                                                 NAT.EC_FLAG_PARITY_ONLY)
            t5 = time.perf_counter()
            assert rc == 0
            segment.pinned_pool.put(out)
            if it >= 2:
                first.append(t1 - t0)
                whole.append(t2 - t0)
                hashes.append(t3 - t0)
                blocking.append(t5 - t4)
                begin.append(tb - t0)
        f, w, h, bl, bg = (float(np.median(x)) for x in (first, whole, hashes, blocking, begin))
        res[hashed] = (f, w, h, bl)
        tag = "hash_pieces=True" if hashed else "no hashes"
        print(f"streamed upload, {tag} (chunk {'library default' if not chunk else chunk}): first parity byte after "
              f"{f * 1e3:.3f} ms ({100 * f / w:.1f} % of the segment), whole segment {w * 1e3:.2f} ms = "
              f"{SEG / w / 2**30:.2f} GiB/s payload, {(SEG + parity_bytes) / w / 1e9:.1f} GB/s PCIe"
              + (f"; all piece hashes after {h * 1e3:.2f} ms" if hashed else "")
              + f"; pad + ec_upload_begin returned after {bg * 1e3:.3f} ms")
        print(f"  blocking ec_encode_segments_host{'_hashed' if hashed else ''} (parity only): {bl * 1e3:.2f} ms = "
              f"{SEG / bl / 2**30:.2f} GiB/s payload; streamed / blocking whole-segment time {w / bl:.3f}")
    print(f"hashed / unhashed streamed: first byte {res[True][0] / res[False][0]:.3f}, whole segment "
          f"{res[True][1] / res[False][1]:.3f}, hashes ready / unhashed whole segment {res[True][2] / res[False][1]:.3f}")
    be.close()


if __name__ == "__main__":
    main()
