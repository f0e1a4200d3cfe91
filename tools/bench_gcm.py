#!/usr/bin/env python3
"""Developer measurement for SURVEY.md §8f row 4 (segment encryption):
AES-256-GCM seal and open of 64 MiB plaintext segments in storj's framing
(9059 blocks of 7408 B -> 7424 B, BlockSize 29*256), inputs resident in HBM,
a batch of NSEG segments with their own keys and nonces per launch.

Prints one JSON line: µs per segment and GB/s of plaintext for seal and open,
the kernel's per-block work, and a CPU baseline: the oracle (OpenSSL
AES-256-GCM with AES-NI, one block per call, storj framing) on 16 host
threads over a bounded sample.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from uplink_amd import encryption as E  # noqa: E402

IB, NB = 7408, 9059


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nseg", type=int, default=8)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--cpu-sample-s", type=float, default=5.0)
    ap.add_argument("--lib", default=None, help="another build of the library (A/B)")
    args = ap.parse_args()
    if args.lib:
        from uplink_amd import _native
        _native.load(args.lib)  # (the process's library from here on)
    torch.cuda.set_device(0)
    nseg = args.nseg
    rng = np.random.default_rng(3)
    keys = [rng.integers(0, 256, 32, dtype=np.uint8).tobytes() for _ in range(nseg)]
    nonces = b"".join(E.nonce_for_position(0, i)[:12] for i in range(nseg))
    g = torch.Generator(device="cuda").manual_seed(2)
    plain = torch.randint(0, 256, (nseg, NB * IB), dtype=torch.uint8, device="cuda", generator=g)
    ct = torch.empty((nseg, NB * (IB + 16)), dtype=torch.uint8, device="cuda")
    back = torch.empty_like(plain)
    status = torch.zeros(nseg, dtype=torch.int32, device="cuda")
    d_keys = E.prepare_keys(keys)
    d_nonces = torch.from_numpy(np.frombuffer(nonces, dtype=np.uint8).copy()).cuda()
    st = torch.cuda.Stream()

    def seal():
        E.seal_segments(plain, nseg, NB, IB, d_keys, d_nonces, ct, stream=st)

    def open_():
        E.open_segments(ct, nseg, NB, IB, d_keys, d_nonces, back, status, stream=st)

    def timed(f):
        t_end = time.time() + 0.3
        while time.time() < t_end:
            f()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(st):
            e0.record(st)
            for _ in range(args.iters):
                f()
            e1.record(st)
        e1.synchronize()
        return e0.elapsed_time(e1) / 1e3 / args.iters

    t_seal = timed(seal)
    t_open = timed(open_)
    torch.cuda.synchronize()
    assert torch.equal(back, plain) and status.max().item() == -1
    pbytes = nseg * NB * IB
    out = {
        "metric": "aes256gcm_segment_GBps", "unit": "GB/s", "dtype": "u32",
        "config": {"workload": f"AES-256-GCM of {nseg} x 64 MiB plaintext segments, {NB} blocks of {IB} B "
                               "(storj BlockSize 7424), own key and nonce per segment, resident in HBM"},
        "seal": {"us_per_segment": t_seal / nseg * 1e6, "GBps": pbytes / t_seal / 1e9},
        "open": {"us_per_segment": t_open / nseg * 1e6, "GBps": pbytes / t_open / 1e9},
        "hbm_frac_seal": (pbytes * 2 + nseg * NB * 16) / t_seal / 8e12,
    }
    from oracle import aesgcm as oa
    host = plain[0, :2000 * IB].cpu().numpy()
    sink = np.zeros((2000, IB + 16), dtype=np.uint8)  # pre-faulted: time the cipher, not page faults
    done, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < args.cpu_sample_s:
        oa.encrypt_blocks(keys[0], nonces[:12], host, IB, threads=args.cpu_threads, out=sink)
        done += 2000
    dt = time.perf_counter() - t0
    out["cpu_baseline"] = {"value": done * IB / dt / 1e9, "unit": "GB/s", "cores": args.cpu_threads,
                           "kind": "port", "sample": f"{done} blocks of {IB} B sealed in {dt:.1f} s (OpenSSL, AES-NI)"}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
