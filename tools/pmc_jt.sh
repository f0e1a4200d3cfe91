#!/bin/bash
# Developer script: SQ / SQC counters of a rebuild experiment variant
# (tools/exp/dec_jump3.hip; VARIANTS = variant indices, SET = share set).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmcjt
BIN=${BIN:-tools/exp/bin/dec_jump3}
for v in ${VARIANTS:-1}; do
  timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_IFETCH SQ_IFETCH_LEVEL --kernel-trace --output-format csv -d gpurun_out/pmcjt/a$v -o run -- $BIN $v > gpurun_out/pmcjt/a$v.log 2>&1 || exit 1
  timeout -s KILL 60 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmcjt/b$v -o run -- $BIN $v > gpurun_out/pmcjt/b$v.log 2>&1 || exit 1
  timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS --kernel-trace --output-format csv -d gpurun_out/pmcjt/c$v -o run -- $BIN $v > gpurun_out/pmcjt/c$v.log 2>&1 || exit 1
done
echo done
