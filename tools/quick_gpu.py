"""Developer probe: parity + timing of the stripe kernels on one GPU.

Not part of the product; used during development to check kernels against
the oracle and time them (python tools/quick_gpu.py).
"""
import ctypes
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle as O  # noqa: E402
from uplink_amd import _native  # noqa: E402

L = _native.load()


def mk(k, n, ess):
    h = ctypes.c_void_p()
    rc = L.ec_create(k, n, ess, ctypes.byref(h))
    assert rc == 0, rc
    return h


def encode_dev(h, seg_t, nseg, nstripes, pieces_t, flags=0):
    rc = L.ec_encode_segments(h, seg_t.data_ptr(), nseg, nstripes, pieces_t.data_ptr(), flags,
                              torch.cuda.current_stream().cuda_stream)
    assert rc == 0, rc


def rebuild_dev(h, nums, piece_ptrs, nstripes, out_t):
    arr = (ctypes.c_int * len(nums))(*nums)
    ptrs = (ctypes.c_void_p * len(piece_ptrs))(*piece_ptrs)
    rc = L.ec_rebuild_segments(h, len(nums), arr, ptrs, nstripes, out_t.data_ptr(),
                               torch.cuda.current_stream().cuda_stream)
    assert rc == 0, rc


def check(k, n, ess, nstripes, iters=20):
    h = mk(k, n, ess)
    print(f"RS({k},{n}) ess={ess} stripes={nstripes} kernel={L.ec_encode_kernel_name(h).decode()}", flush=True)
    rng = np.random.default_rng(1)
    seg = rng.integers(0, 256, nstripes * k * ess, dtype=np.uint8)
    plen = nstripes * ess
    t0 = time.time()
    ref = O.FEC(k, n).encode_segment(seg, ess, threads=8)
    print(f"  oracle encode {time.time()-t0:.2f}s", flush=True)
    seg_t = torch.from_numpy(seg).cuda()
    pieces_t = torch.zeros(n * plen, dtype=torch.uint8, device="cuda")
    encode_dev(h, seg_t, 1, nstripes, pieces_t)
    torch.cuda.synchronize()
    got = pieces_t.cpu().numpy().reshape(n, plen)
    bad = np.nonzero((got != ref).any(axis=1))[0]
    print("  encode parity:", "OK" if len(bad) == 0 else f"MISMATCH rows {bad[:10]}", flush=True)
    # decode from the last k pieces (all parity when n-k >= k)
    nums = list(range(n - k, n))
    out_t = torch.zeros(nstripes * k * ess, dtype=torch.uint8, device="cuda")
    base = pieces_t.data_ptr()
    rebuild_dev(h, nums, [base + i * plen for i in nums], nstripes, out_t)
    torch.cuda.synchronize()
    ok = np.array_equal(out_t.cpu().numpy(), seg)
    print("  rebuild from", nums[0], "..", nums[-1], ":", "OK" if ok else "MISMATCH", flush=True)
    rs = np.random.default_rng(29)
    nums2 = sorted(rs.choice(n, k, replace=False).tolist())
    out_t.zero_()
    rebuild_dev(h, nums2, [base + i * plen for i in nums2], nstripes, out_t)
    torch.cuda.synchronize()
    ok2 = np.array_equal(out_t.cpu().numpy(), seg)
    print("  rebuild random subset:", "OK" if ok2 else "MISMATCH", flush=True)
    # timing
    s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        encode_dev(h, seg_t, 1, nstripes, pieces_t)
    torch.cuda.synchronize()
    s0.record()
    for _ in range(iters):
        encode_dev(h, seg_t, 1, nstripes, pieces_t)
    s1.record()
    torch.cuda.synchronize()
    te = s0.elapsed_time(s1) / iters * 1e3
    spad = nstripes * k * ess
    print(f"  encode {te:.1f} us  {spad/te/1e3:.1f} GB/s payload  "
          f"{spad*(1+n/k)/te/1e3:.1f} GB/s algorithmic", flush=True)
    for nn, lab in ((nums, "parity-set"), (nums2, "random-set")):
        ptrs = [base + i * plen for i in nn]
        rebuild_dev(h, nn, ptrs, nstripes, out_t)
        torch.cuda.synchronize()
        s0.record()
        for _ in range(iters):
            rebuild_dev(h, nn, ptrs, nstripes, out_t)
        s1.record()
        torch.cuda.synchronize()
        td = s0.elapsed_time(s1) / iters * 1e3
        print(f"  rebuild[{lab}] {td:.1f} us  {spad/td/1e3:.1f} GB/s payload  {2*spad/td/1e3:.1f} GB/s alg",
              flush=True)
    L.ec_destroy(h)


if __name__ == "__main__":
    torch.cuda.init()
    check(29, 80, 256, 9040)
    check(20, 60, 4096, 820)
    check(4, 10, 256, 1025, iters=50)
    check(30, 60, 1024, 257, iters=20)
    check(3, 7, 1024, 2, iters=5)
