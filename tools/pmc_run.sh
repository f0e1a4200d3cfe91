#!/bin/bash
# Developer script: PMC passes (separate runs, kernel-trace only) for bench.py
# and the decode experiment.  Output under gpurun_out/pmc/.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/pmc/bench_$C -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmc/bench_$C.log 2>&1
done
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --kernel-trace --output-format csv -d gpurun_out/pmc/dec_sq -o run -- tools/exp/bin/decode_exp 0 > gpurun_out/pmc/dec_sq.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_SMEM SQ_WAIT_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_ANY --kernel-trace --output-format csv -d gpurun_out/pmc/dec_sq2 -o run -- tools/exp/bin/decode_exp 0 > gpurun_out/pmc/dec_sq2.log 2>&1 || true
echo done
