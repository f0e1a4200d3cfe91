#!/usr/bin/env python3
"""Developer measurement: the device-resident segment chain of
uplink_amd/pipeline.py on a batch of 64 MiB plaintext segments, RS(29,80).

  upload    pad + AES-256-GCM seal (into the padded RS input) + PadReader +
            encode all 80 pieces + BLAKE3 of every piece
  download  rebuild from 29 parity pieces + AES-256-GCM open (tag check)

Prints one JSON line: µs per segment and plaintext GiB/s for each direction,
inputs resident in HBM.  Never the bench.py value."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from uplink_amd import eestream, encryption as E, pipeline  # noqa: E402

K, N, PLAIN, NSEG, ITERS = 29, 80, 64 * 2**20, 8, 10


def main():
    torch.cuda.set_device(0)
    sch = eestream.RSScheme(eestream.new_fec(K, N), 256)
    p = pipeline.DevicePipeline(sch, PLAIN)
    rng = np.random.default_rng(1)
    keys = [rng.integers(0, 256, 32, dtype=np.uint8).tobytes() for _ in range(NSEG)]
    d_keys = p.prepare_keys(keys)
    d_nonces = p.nonces_tensor([E.nonce_for_position(0, i) for i in range(NSEG)])
    d_plain, d_enc, d_pieces, d_hashes = p.buffers(NSEG)
    d_plain.random_(0, 256)
    d_out = torch.empty_like(d_plain)
    d_status = torch.zeros(NSEG, dtype=torch.int32, device="cuda")
    nums = list(range(N - K, N))
    st = torch.cuda.Stream()

    def up():
        p.upload(d_plain, NSEG, d_keys, d_nonces, d_enc, d_pieces, d_hashes, stream=st)

    def down():
        p.download(nums, d_pieces, NSEG, d_keys, d_nonces, d_enc, d_out, d_status, stream=st)

    def timed(f):
        t_end = time.time() + 0.3
        while time.time() < t_end:
            f()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(st):
            e0.record(st)
            for _ in range(ITERS):
                f()
            e1.record(st)
        e1.synchronize()
        return e0.elapsed_time(e1) / 1e3 / ITERS

    t_up, t_down = timed(up), timed(down)
    torch.cuda.synchronize()
    assert d_status.max().item() == -1 and torch.equal(d_out[:, :PLAIN], d_plain[:, :PLAIN])
    print(json.dumps({
        "metric": "device-resident segment chain, RS(29,80) + AES-256-GCM + BLAKE3", "unit": "GiB/s plaintext",
        "segments_per_launch": NSEG, "plain_bytes": PLAIN,
        "upload": {"us_per_segment": t_up / NSEG * 1e6, "GiBps": NSEG * PLAIN / t_up / 2**30},
        "download": {"us_per_segment": t_down / NSEG * 1e6, "GiBps": NSEG * PLAIN / t_down / 2**30},
    }))


if __name__ == "__main__":
    main()
