"""Experiment: PCIe copy rates on the box with pinned host memory: H2D alone,
D2H alone, and both at once on two streams (is the link full duplex for us?)."""
import time

import torch

N = 256 * 2**20
h_in = torch.empty(N, dtype=torch.uint8).pin_memory()
h_out = torch.empty(N, dtype=torch.uint8).pin_memory()
d_a = torch.empty(N, dtype=torch.uint8, device="cuda")
d_b = torch.empty(N, dtype=torch.uint8, device="cuda")
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def run(h2d, d2h, reps=10):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        if h2d:
            with torch.cuda.stream(s1):
                d_a.copy_(h_in, non_blocking=True)
        if d2h:
            with torch.cuda.stream(s2):
                h_out.copy_(d_b, non_blocking=True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    return reps * N * (h2d + d2h) / dt / 1e9


for _ in range(2):
    print(f"H2D alone {run(1, 0):.1f} GB/s   D2H alone {run(0, 1):.1f} GB/s   both at once {run(1, 1):.1f} GB/s total")
