#!/usr/bin/env python3
"""Experiment (GPU box): the encode through the runtime-matrix kernel with
straight-line code (ec_set_body(EC_BODY_STRAIGHT_LINE): 5-8 waves per
workgroup, one pass for up to 64 parity rows) against the compile-time
encoder (EC_BODY_JUMP_TABLE), full and parity-only, 16 x 64 MiB segments.
python tools/exp/sl_encode_probe.py [k n ...]"""
import ctypes
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

CONFIGS = ((29, 80), (20, 50), (30, 60), (50, 80), (20, 60))


def child(configs):
    import numpy as np
    import torch
    from oracle import oracle as O
    from uplink_amd import _native
    L = _native.load()
    s = torch.cuda.current_stream().cuda_stream
    nseg, ess = 16, 256
    for (k, n), body in [(c, b) for c in configs for b in (_native.EC_BODY_JUMP_TABLE, _native.EC_BODY_STRAIGHT_LINE)]:
        stripes = ((64 << 20) + 4 + k * ess - 1) // (k * ess)
        spad, plen = stripes * k * ess, stripes * ess
        ctx = ctypes.c_void_p()
        assert L.ec_create(k, n, ess, ctypes.byref(ctx)) == 0
        assert L.ec_set_body(ctx, body) == 0
        segs = torch.randint(0, 256, (nseg, spad), dtype=torch.uint8, device="cuda")
        res = {"k": k, "n": n, "kernel": L.ec_encode_kernel_name(ctx).decode()}
        for name, flags, rows in (("full", 0, n), ("parity", _native.EC_FLAG_PARITY_ONLY, n - k)):
            pcs = torch.empty((nseg, rows, plen), dtype=torch.uint8, device="cuda")

            def enc():
                assert L.ec_encode_segments(ctx, segs.data_ptr(), nseg, stripes, pcs.data_ptr(), flags, s) == 0
            for _ in range(5):
                enc()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                enc()
            e1.record()
            e1.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / 10 / nseg
            ref = O.FEC(k, n).encode_segment(segs[3, :64 * k * ess].cpu().numpy(), ess, threads=4)
            got = pcs[3, :, :64 * ess].cpu().numpy()
            ok = bool(np.array_equal(got, ref if rows == n else ref[k:]))
            byt = spad * (1 + rows / k)
            res[name] = {"us_per_segment": round(us, 2), "TBps": round(byt / us / 1e6, 3), "ok": ok,
                         "body": L.ec_last_body(ctx)}
            del pcs
        print(json.dumps(res), flush=True)
        del segs
        L.ec_destroy(ctx)


if __name__ == "__main__":
    a = [int(x) for x in sys.argv[1:]]
    child(list(zip(a[0::2], a[1::2])) or CONFIGS)
