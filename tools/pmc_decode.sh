#!/bin/bash
# Developer script (GPU box): SQ counter passes (kernel trace only, one pass per
# group) over Decode with detection at k+20 (tools/exp/ab_decode_rows.py 20),
# summarised by tools/pmc_sq_summary.py.  Usage: pmc_decode.sh OUTDIR
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05/pmc_decode}
mkdir -p $O
i=0
for G in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_CYCLES" \
         "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_IFETCH SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"; do
  timeout -s KILL 120 rocprofv3 --pmc $G --kernel-trace --output-format csv -d $O/p$i -o run -- python3 tools/exp/ab_decode_rows.py 20 > $O/p$i.log 2>&1
  i=$((i+1))
done
python3 tools/pmc_sq_summary.py $O $O/sq_summary.json > $O/sq_summary.txt
echo done
