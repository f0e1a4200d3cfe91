#!/usr/bin/env python3
"""A/B of the straight-line split past 32 rows (UPLINK_SL_WIDE_ROWS_PER_WAVE,
read once per process): Decode with detection at k+1..k+20 on whole RS(29,80)
64 MiB segments, bench.py's informational leg.  Run once per setting;
args: [--lib=PATH] the extra-share counts (default 1 4 10 20)."""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
from uplink_amd import _native  # noqa: E402

torch.cuda.set_device(0)
args = sys.argv[1:]
lib = None
if args and args[0].startswith("--lib="):
    lib = args.pop(0)[len("--lib="):]
extras = tuple(int(x) for x in args) or (1, 4, 10, 20)
L = _native.load(lib) if lib else _native.load()
res = bench.decode_with_detection(L, torch.device("cuda", 0), torch.cuda.current_stream().cuda_stream, extras=extras)
print(json.dumps({"rows_per_wave": os.environ.get("UPLINK_SL_WIDE_ROWS_PER_WAVE", "default"), "lib": lib,
                  "depth": os.environ.get("UPLINK_EC_REBUILD_DEPTH", "default"),
                  **{k: v for k, v in res.items() if k != "note"}}))
