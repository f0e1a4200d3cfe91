#!/bin/bash
# Developer script: one PMC pass (LDS / VALU activity) over tools/bench_gcm.py on the GPU box
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/gcm/pmc
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O -o run -- python3 tools/bench_gcm.py --iters 3 --cpu-sample-s 0.2 > $O/log 2>&1
echo done
