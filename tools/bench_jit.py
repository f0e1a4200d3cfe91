#!/usr/bin/env python3
"""Run-time-compiled encoders: how long the hiprtc compilation of one (k, n)
takes (cold: empty cache directory; warm: a second process reading the
cached code object), and the encode speed of the compiled kernel against the
runtime-matrix kernel it replaces while it compiles.  One JSON line per
(k, n).  Run on a GPU box:  python tools/bench_jit.py [k n ...]
"""
import ctypes
import json
import os
import subprocess
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)


def child(k, n):
    """In a fresh process: time ec_prepare_encoder(wait) and the encodes."""
    import torch
    from uplink_amd import _native
    L = _native.load()
    dev = torch.device("cuda", 0)
    ctx = ctypes.c_void_p()
    assert L.ec_create(k, n, 256, ctypes.byref(ctx)) == 0
    stripes = (64 << 20) // (k * 256) + 1
    nseg = 4
    segs = torch.randint(0, 256, (nseg, stripes * k * 256), dtype=torch.uint8, device=dev)
    pieces = torch.empty((nseg, n, stripes * 256), dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream().cuda_stream

    def enc():
        assert L.ec_encode_segments(ctx, segs.data_ptr(), nseg, stripes, pieces.data_ptr(), 0, s) == 0

    def timed(it=10):
        enc()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(it):
            enc()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / it / nseg

    before = L.ec_encode_kernel_name(ctx).decode()
    t_generic = timed() if before == "generic" else None
    ref = pieces.clone() if t_generic is not None else None
    t0 = time.perf_counter()
    ready = L.ec_prepare_encoder(ctx, 1)
    t_prep = time.perf_counter() - t0
    after = L.ec_encode_kernel_name(ctx).decode()
    t_special = timed()
    same = bool(torch.equal(pieces, ref)) if ref is not None else None
    seg_bytes = stripes * k * 256 * (1 + n / k)
    print(json.dumps({"k": k, "n": n, "kernel_before": before, "kernel_after": after, "ready": ready,
                      "prepare_wait_s": round(t_prep, 3),
                      "generic_us_per_segment": None if t_generic is None else round(t_generic, 2),
                      "special_us_per_segment": round(t_special, 2),
                      "special_TBps": round(seg_bytes / t_special / 1e6, 3),
                      "identical_pieces": same}), flush=True)


def main(pairs):
    with tempfile.TemporaryDirectory() as cache:
        env = dict(os.environ, UPLINK_EC_JIT_CACHE=cache)
        for k, n in pairs:
            for run in ("cold", "warm"):
                r = subprocess.run([sys.executable, __file__, "--child", str(k), str(n)], env=env,
                                   capture_output=True, text=True, timeout=600)
                line = [x for x in r.stdout.splitlines() if x.startswith("{")]
                if r.returncode or not line:
                    print(json.dumps({"k": k, "n": n, "run": run, "rc": r.returncode, "stderr": r.stderr[-800:]}))
                    continue
                d = json.loads(line[-1])
                d["run"] = run
                print(json.dumps(d), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        child(int(sys.argv[2]), int(sys.argv[3]))
    else:
        a = [int(x) for x in sys.argv[1:]] or [16, 40, 37, 50, 64, 96, 10, 100]
        main(list(zip(a[0::2], a[1::2])))
