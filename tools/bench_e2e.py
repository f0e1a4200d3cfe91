"""End-to-end rate with host buffers (BASELINE configs[4]):
segments start in pinned host memory and end there; H2D, kernel and D2H of
consecutive segments overlap on 3 HIP streams (hipMemcpyAsync via torch
non_blocking copies on pinned tensors).  PCIe-inclusive; reported in
DESIGN.md, never as bench.py's value.

  python tools/bench_e2e.py [--k 20 --n 60 --ess 4096 --segments 12]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from uplink_amd import eestream  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=20)
    ap.add_argument("--n", type=int, default=60)
    ap.add_argument("--ess", type=int, default=4096)
    ap.add_argument("--segments", type=int, default=12)
    ap.add_argument("--mode", default="mixed", choices=["mixed", "encode", "decode", "encode-parity"])
    ap.add_argument("--slots", type=int, default=3)
    ap.add_argument("--reps", type=int, default=5, help="capi: timed repetitions (median reported)")
    ap.add_argument("--api", default="torch", choices=["torch", "capi"],
                    help="torch: pipeline orchestrated here; capi: ec_*_segments_host in the library")
    args = ap.parse_args()
    if args.api == "capi":
        return capi(args)
    k, n, ess = args.k, args.n, args.ess
    raw = 64 * 2**20
    stripes = (raw + 4 + k * ess - 1) // (k * ess)
    spad = stripes * k * ess
    plen = stripes * ess
    sch = eestream.RSScheme(eestream.new_fec(k, n), ess)
    codec = eestream.SegmentCodec(sch)
    dev = torch.device("cuda", 0)
    nseg = args.segments
    rng = np.random.default_rng(1)
    # pinned host buffers: segments in, pieces out (encode); pieces in, segment out (decode)
    h_seg = torch.empty((nseg, spad), dtype=torch.uint8, pin_memory=True)
    h_seg.copy_(torch.from_numpy(rng.integers(0, 256, (nseg, spad), dtype=np.uint8)))
    rows = n - k if args.mode == "encode-parity" else n
    h_pieces = torch.empty((nseg, rows, plen), dtype=torch.uint8, pin_memory=True)
    h_out = torch.empty((nseg, spad), dtype=torch.uint8, pin_memory=True)
    dec_nums = list(range(n - k, n))
    # decode inputs: valid pieces of each segment (encoded once up front on the GPU)
    h_dec_in = torch.empty((nseg, k, plen), dtype=torch.uint8, pin_memory=True)
    tmp_p = torch.empty((1, n, plen), dtype=torch.uint8, device=dev)
    for g in range(nseg):
        codec.encode_segments(h_seg[g].to(dev), 1, stripes, tmp_p)
        h_dec_in[g].copy_(tmp_p[0, n - k:].cpu())
    torch.cuda.synchronize()
    S = args.slots
    streams = [torch.cuda.Stream(dev) for _ in range(S)]
    d_seg = [torch.empty(spad, dtype=torch.uint8, device=dev) for _ in range(S)]
    d_pieces = [torch.empty((rows, plen), dtype=torch.uint8, device=dev) for _ in range(S)]
    d_dec_in = [torch.empty((k, plen), dtype=torch.uint8, device=dev) for _ in range(S)]
    d_out = [torch.empty(spad, dtype=torch.uint8, device=dev) for _ in range(S)]

    def job(g, s):
        st = streams[s]
        kind = args.mode
        if kind == "mixed":
            kind = "encode" if g % 2 == 0 else "decode"
        with torch.cuda.stream(st):
            if kind in ("encode", "encode-parity"):
                d_seg[s].copy_(h_seg[g], non_blocking=True)
                codec.encode_segments(d_seg[s], 1, stripes, d_pieces[s], parity_only=(kind == "encode-parity"),
                                      stream=st)
                h_pieces[g].copy_(d_pieces[s], non_blocking=True)
                return spad, spad + rows * plen
            d_dec_in[s].copy_(h_dec_in[g], non_blocking=True)
            base = d_dec_in[s].data_ptr()
            codec.rebuild_segments(dec_nums, [base + i * plen for i in range(k)], stripes, d_out[s], stream=st)
            h_out[g].copy_(d_out[s], non_blocking=True)
            return spad, 2 * spad

    for g in range(S):  # warm-up
        job(g, g % S)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    payload = pcie = 0
    for g in range(nseg):
        p, b = job(g, g % S)
        payload += p
        pcie += b
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    # correctness spot check
    ok = True
    for g in range(nseg):
        kind = args.mode if args.mode != "mixed" else ("encode" if g % 2 == 0 else "decode")
        if kind == "decode":
            ok &= bool(torch.equal(h_out[g], h_seg[g]))
        elif kind == "encode":
            ok &= bool(torch.equal(h_pieces[g, :k].reshape(-1), h_seg[g].view(stripes, k, ess).transpose(0, 1).reshape(-1)))
    print(json.dumps({"config": f"RS({k},{n}) ess={ess} 64MiB segments, mode={args.mode}, {nseg} segments, "
                                f"{S} streams, pinned host buffers",
                      "payload_GiBps": round(payload / wall / 2**30, 2), "pcie_GBps": round(pcie / wall / 1e9, 2),
                      "ms_per_segment": round(wall / nseg * 1e3, 3), "verified": ok}))


def capi(args):
    """The library's own host pipeline (ec_encode_segments_host /
    ec_rebuild_segments_host) on ec_host_alloc'd pinned buffers."""
    import ctypes
    from uplink_amd import _native
    lib = _native.load()
    k, n, ess = args.k, args.n, args.ess
    stripes = (64 * 2**20 + 4 + k * ess - 1) // (k * ess)
    spad, plen = stripes * k * ess, stripes * ess
    sch = eestream.RSScheme(eestream.new_fec(k, n), ess)
    nseg = args.segments
    rows = n - k if args.mode == "encode-parity" else n

    def pinned(nbytes):
        p = lib.ec_host_alloc(nbytes)
        assert p, "ec_host_alloc failed"
        return p, np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(p))
    ps, segs = pinned(nseg * spad)
    segs[:] = np.random.default_rng(1).integers(0, 256, nseg * spad, dtype=np.uint8)
    pp, pieces = pinned(nseg * n * plen)
    po, out = pinned(nseg * spad)
    flags = _native.EC_FLAG_PARITY_ONLY if args.mode == "encode-parity" else 0
    assert lib.ec_encode_segments_host(sch.ctx, ps, nseg, stripes, pp, 0) == 0  # warm + decode inputs
    nums = list(range(n - k, n))
    c_nums = (ctypes.c_int * k)(*nums)
    c_ptrs = (ctypes.c_void_p * k)(*[pp + i * plen for i in nums])
    res = {}

    def run(mode):
        if mode.startswith("encode"):
            return lib.ec_encode_segments_host(sch.ctx, ps, nseg, stripes, pp, flags), nseg * (spad + rows * plen)
        return lib.ec_rebuild_segments_host(sch.ctx, k, c_nums, c_ptrs, stripes, nseg, n * plen, po), nseg * 2 * spad

    modes = ["encode", "decode"] if args.mode == "mixed" else [args.mode]
    for mode in modes:  # untimed: plans, pipeline buffers, first-touch of the pinned pages
        assert run(mode)[0] == 0
    walls = {m: [] for m in modes}
    for _ in range(args.reps):
        for mode in modes:
            t0 = time.perf_counter()
            rc, pcie = run(mode)
            walls[mode].append(time.perf_counter() - t0)
            assert rc == 0, rc
            res[mode] = (nseg * spad, pcie, sorted(walls[mode])[len(walls[mode]) // 2])  # median
    ok = bool(np.array_equal(out, segs)) if "decode" in res else True
    pay = sum(v[0] for v in res.values())
    pc = sum(v[1] for v in res.values())
    wall = sum(v[2] for v in res.values())
    print(json.dumps({"config": f"RS({k},{n}) ess={ess} 64MiB segments, mode={args.mode}, {nseg} segments, "
                                f"library host pipeline (ec_*_segments_host, 3 streams, ec_host_alloc pinned), "
                                f"median of {args.reps} after a warm-up call",
                      "payload_GiBps": round(pay / wall / 2**30, 2), "pcie_GBps": round(pc / wall / 1e9, 2),
                      "ms_per_segment": round(wall / (nseg * len(res)) * 1e3, 3), "verified": ok}))
    for p in (ps, pp, po):
        lib.ec_host_free(p)


if __name__ == "__main__":
    main()
