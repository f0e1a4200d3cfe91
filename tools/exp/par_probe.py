"""Experiment: full (80 pieces) vs parity-only (51 pieces) encode launch time,
alternating, same buffers warm."""
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
full = torch.empty((B, N, ST * ESS), dtype=torch.uint8, device="cuda")
par = torch.empty((B, N - K, ST * ESS), dtype=torch.uint8, device="cuda")
s = torch.cuda.current_stream().cuda_stream


def run(buf, flags, n=20):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        L.ec_encode_segments(h, segs.data_ptr(), B, ST, buf.data_ptr(), flags, s)
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


for _ in range(30):
    run(full, 0, 4)
for rep in range(3):
    tf = run(full, 0)
    tp = run(par, _native.EC_FLAG_PARITY_ONLY)
    print(f"full {tf:.1f} us  parity-only {tp:.1f} us per launch of {B} segments")
