#!/bin/bash
# Developer script (GPU box): the round's measurement set for the final tree,
# under gpurun_out/$1 (default r02/final): the default bench line, the same
# bench under rocprofv3 --kernel-trace --stats (kernel durations to compare
# with the bench's HIP events), the HBM traffic PMC passes (FETCH_SIZE /
# WRITE_SIZE, separate runs) and the SQ activity passes.  Each GPU step has
# its own time limit; the script stops at the first failure.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r02/final}
mkdir -p $O $O/pmc_sq
timeout -k 10 400 python3 bench.py > $O/bench.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu-baseline > $O/bench_under_rocprof.log 2>&1
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/pmc_$C -o run -- python3 bench.py --steps 3 --warmup 1 --settle-s 0 --no-cpu-baseline --no-other-configs > $O/pmc_$C.log 2>&1
done
python3 tools/pmc_traffic.py $O/pmc_FETCH_SIZE $O/pmc_WRITE_SIZE $O/pmc_traffic.json
i=0
for G in "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE" \
         "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_IFETCH SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES"; do
  timeout -s KILL 200 rocprofv3 --pmc $G --kernel-trace --output-format csv -d $O/pmc_sq/p$i -o run -- python3 bench.py --steps 8 --warmup 4 --settle-s 0 --no-cpu-baseline --no-other-configs > $O/pmc_sq/p$i.log 2>&1
  i=$((i+1))
done
echo done
