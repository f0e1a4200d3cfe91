#!/bin/bash
# Developer script (GPU box): instruction-cache counters (SQC_ICACHE_*, SQ
# block) over the RS(29,80) bench launches, one rocprofv3 pass, under
# gpurun_out/$1 (default r03/icache).  Optional second argument: another
# libuplink_ec.so (bench.py --lib) for an A/B.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r03/icache}
mkdir -p $O
LIB=${2:+--lib $2}
timeout -s KILL 200 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_INSTS_VALU SQ_WAVE_CYCLES --kernel-trace --output-format csv -d $O/pmc -o run -- python3 bench.py --steps 4 --warmup 2 --settle-s 0 --no-cpu-baseline --no-other-configs $LIB > $O/pmc.log 2>&1
python3 tools/pmc_sq_summary.py $O/pmc $O/icache_summary.json > /dev/null 2>&1 || true
echo done
