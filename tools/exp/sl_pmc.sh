set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/sl2
mkdir -p $O/pmc
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/exp/sl_prof.py > $O/prof.log 2>&1
i=0
for G in "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE" \
         "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_IFETCH SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES"; do
  timeout -s KILL 90 rocprofv3 --pmc $G --kernel-trace --output-format csv -d $O/pmc/p$i -o run -- python3 tools/exp/sl_prof.py > $O/pmc/p$i.log 2>&1
  i=$((i+1))
done
python3 tools/pmc_sq_summary.py $O/pmc $O/sq_summary.json
timeout -s KILL 60 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS --kernel-trace --output-format csv -d $O/pmc_ic -o run -- python3 tools/exp/sl_prof.py > $O/pmc_ic.log 2>&1
echo done
