"""Developer experiment: time ec_encode_segments back to back vs interleaved
with the rebuild, on torch-allocated buffers (same as bench.py)."""
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
pieces = torch.empty((nb, B.N, B.PIECE), dtype=torch.uint8, device=dev)
out = torch.empty((nb, B.S_PAD), dtype=torch.uint8, device=dev)
s = torch.cuda.current_stream().cuda_stream
sets = B.share_sets()
nums = (ctypes.c_int * B.K)(*sets[0]); base = pieces.data_ptr()
ptrs = (ctypes.c_void_p * B.K)(*[base + j * B.PIECE for j in sets[0]])
enc = lambda: L.ec_encode_segments(ctx, segs.data_ptr(), nb, B.NSTRIPES, pieces.data_ptr(), 0, s)
dec = lambda: L.ec_rebuild_segments_batched(ctx, B.K, nums, ptrs, B.NSTRIPES, nb, B.N * B.PIECE, B.S_PAD, out.data_ptr(), s)
def t(name, fn, it=20):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record(); [fn() for _ in range(it)]; e1.record(); torch.cuda.synchronize()
    print(f"{name:40s} {e0.elapsed_time(e1) * 1e3 / it / nb:8.1f} us/seg", flush=True)
t("encode back-to-back", enc)
t("decode back-to-back", dec)
def pair():
    enc(); dec()
t("encode+decode pairs (sum)", pair)
# encode timed alone but each preceded by a decode
ev = []
for i in range(20):
    dec(); a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
    a.record(); enc(); b.record(); ev.append((a, b))
torch.cuda.synchronize()
print(f"{'encode after decode':40s} {sum(a.elapsed_time(b) for a, b in ev) * 1e3 / 20 / nb:8.1f} us/seg")
