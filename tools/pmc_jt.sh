#!/bin/bash
# Developer script: SQ counters of the jump-table rebuild experiment (tools/exp/dec_jump.hip).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmcjt
BIN=${BIN:-tools/exp/bin/dec_jump}
for v in ${VARIANTS:-1 3}; do
  timeout -k 10 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS --kernel-trace --output-format csv -d gpurun_out/pmcjt/a$v -o run -- $BIN $v > gpurun_out/pmcjt/a$v.log 2>&1 || exit 1
  timeout -k 10 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmcjt/b$v -o run -- $BIN $v > gpurun_out/pmcjt/b$v.log 2>&1 || exit 1
done
echo done
