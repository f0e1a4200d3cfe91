"""Experiment: sustained back-to-back parity-only encodes, per-launch time
(clock/power behaviour of the 8+4 vs 4+4 wave split)."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from uplink_amd import _native  # noqa: E402

L = _native.load()
K, N, ESS, ST, B = 29, 80, 256, 9040, 8
h = ctypes.c_void_p()
assert L.ec_create(K, N, ESS, ctypes.byref(h)) == 0
segs = torch.randint(0, 256, (B, ST * K * ESS), dtype=torch.uint8, device="cuda")
par = torch.empty((B, N - K, ST * ESS), dtype=torch.uint8, device="cuda")
full = torch.empty((B, N, ST * ESS), dtype=torch.uint8, device="cuda")
s = torch.cuda.current_stream().cuda_stream
for name, buf, flags in (("parity-only", par, _native.EC_FLAG_PARITY_ONLY), ("full", full, 0)):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(101)]
    ev[0].record()
    for i in range(100):
        L.ec_encode_segments(h, segs.data_ptr(), B, ST, buf.data_ptr(), flags, s)
        ev[i + 1].record()
    ev[-1].synchronize()
    t = [ev[i].elapsed_time(ev[i + 1]) * 1e3 for i in range(100)]
    print(name, "first 5:", [round(x) for x in t[:5]], "last 50 avg:", round(sum(t[50:]) / 50, 1))
