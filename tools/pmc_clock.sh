#!/bin/bash
# Developer script: effective clock (GRBM_GUI_ACTIVE) of encode variants.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/clk
for v in 0 1 2; do
  timeout -k 10 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES SQ_INSTS_VALU --kernel-trace --output-format csv -d gpurun_out/clk/v$v -o run -- tools/exp/bin/encode_exp $v > gpurun_out/clk/v$v.log 2>&1 || exit 1
done
echo done
