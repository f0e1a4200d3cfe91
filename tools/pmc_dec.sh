#!/bin/bash
# Developer script: SQ counter passes (kernel-trace only, one pass per group)
# over one variant of tools/exp/bin/decode_exp.  Usage: pmc_dec.sh VARIANT TAG
set -e
V=${1:-0}; T=${2:-dec}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc
i=0
for G in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_CYCLES" \
         "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_IFETCH SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"; do
  timeout -k 10 120 rocprofv3 --pmc $G --kernel-trace --output-format csv -d gpurun_out/pmc/${T}_$i -o run -- tools/exp/bin/decode_exp $V > gpurun_out/pmc/${T}_$i.log 2>&1
  i=$((i+1))
done
echo done
