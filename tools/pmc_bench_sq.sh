#!/bin/bash
# Developer script: SQ activity counters of the bench's kernels (one pass each, kernel-trace only)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/pmc_sq
mkdir -p $O
i=0
for G in "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE" \
         "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_IFETCH SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES"; do
  timeout -s KILL 150 rocprofv3 --pmc $G --kernel-trace --output-format csv -d $O/p$i -o run -- python3 bench.py --steps 8 --warmup 4 --settle-s 0 --no-cpu-baseline > $O/p$i.log 2>&1
  i=$((i+1))
done
echo done
