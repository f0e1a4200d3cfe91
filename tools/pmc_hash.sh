#!/bin/bash
# Developer script: BLAKE3 piece-hash measurement on the GPU box:
# bench line, kernel-trace stats, and one PMC pass for the VALU count.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/hash
mkdir -p $O
timeout -k 10 200 python3 tools/bench_hash.py "$@" > $O/bench.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/bench_hash.py --iters 20 --cpu-sample-s 0.5 > $O/prof.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES --kernel-trace --output-format csv -d $O/pmc -o run -- python3 tools/bench_hash.py --iters 3 --cpu-sample-s 0.5 > $O/pmc.log 2>&1
echo done
