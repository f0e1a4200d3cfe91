"""Developer experiment: encode of batch i+1 on one stream concurrently with
the rebuild of batch i on another (double-buffered pieces) vs the two kernels
back to back on one stream."""
import ctypes, os, sys, time
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench as B
from uplink_amd import _native

L = _native.load()
dev = torch.device("cuda", 0)
ctx = ctypes.c_void_p(); assert L.ec_create(B.K, B.N, B.ESS, ctypes.byref(ctx)) == 0
nb = 8
segs = B.padded_segments(nb, 0, dev)
pieces = [torch.empty((nb, B.N, B.PIECE), dtype=torch.uint8, device=dev) for _ in range(2)]
out = torch.empty((nb, B.S_PAD), dtype=torch.uint8, device=dev)
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
sets = B.share_sets()
nums = [(ctypes.c_int * B.K)(*s) for s in sets]
def ptrs(p, s): return (ctypes.c_void_p * B.K)(*[p.data_ptr() + j * B.PIECE for j in s])
P = [[ptrs(p, s) for s in sets] for p in pieces]
def enc(buf, st): assert L.ec_encode_segments(ctx, segs.data_ptr(), nb, B.NSTRIPES, pieces[buf].data_ptr(), 0, st.cuda_stream) == 0
def dec(buf, i, st): assert L.ec_rebuild_segments_batched(ctx, B.K, nums[i % 8], P[buf][i % 8], B.NSTRIPES, nb, B.N * B.PIECE, B.S_PAD, out.data_ptr(), st.cuda_stream) == 0
def seq(steps):
    for i in range(steps):
        enc(0, s1); dec(0, i, s1)
def pipe(steps):
    enc(0, s1)
    for i in range(steps):
        ev = torch.cuda.Event(); ev.record(s1)
        s2.wait_event(ev)
        enc((i + 1) % 2, s1)          # next batch
        dec(i % 2, i, s2)             # this batch
        ev2 = torch.cuda.Event(); ev2.record(s2)
        s1.wait_event(ev2)            # next encode may not overwrite what the rebuild reads
def timeit(name, fn, steps=40):
    for _ in range(2):
        fn(40); torch.cuda.synchronize()
    t0 = time.perf_counter(); fn(steps); torch.cuda.synchronize(); t = time.perf_counter() - t0
    print(f"{name:30s} {t / steps * 1e6 / nb:7.1f} us per segment pair  {nb * steps * B.S_PAD / 2**30 / t:7.1f} GiB/s", flush=True)
t_end = time.perf_counter() + 0.5
while time.perf_counter() < t_end: seq(8); torch.cuda.synchronize()
timeit("sequential (one stream)", seq)
timeit("pipelined (two streams)", pipe)
timeit("sequential (one stream)", seq)
timeit("pipelined (two streams)", pipe)
