#!/bin/bash
# Developer script (GPU box): GPU parity of the encoder, then the bench A/B of
# library builds (A B C A B C).  bash tools/exp/r3_enc_ab.sh OUT LIB_A LIB_B [LIB_C]
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; shift
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_parity.log 2>&1
for i in 1 2; do
  n=0
  for L in "$@"; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-other-configs --lib $L > $O/v${n}_$i.log 2>&1
    n=$((n+1))
  done
done
echo done
