#!/bin/bash
# Developer script: HBM traffic PMC passes (separate runs, kernel-trace only)
# of bench.py; output under gpurun_out/pmc/, summary -> gpurun_out/pmc/pmc_traffic.json
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/pmc/bench_$C -o run -- python3 bench.py --steps 3 --warmup 1 --settle-s 0 --no-cpu-baseline > gpurun_out/pmc/bench_$C.log 2>&1
done
python3 tools/pmc_traffic.py gpurun_out/pmc/bench_FETCH_SIZE gpurun_out/pmc/bench_WRITE_SIZE gpurun_out/pmc/pmc_traffic.json
echo done
