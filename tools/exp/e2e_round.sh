#!/bin/bash
# PCIe-inclusive host pipelines through the C-ABI (GPU box), every mode for
# C5 RS(20,60) ess 4096 and RS(29,80) ess 256:  bash tools/exp/e2e_round.sh OUTDIR
set -e
O=$1
mkdir -p $O
for m in mixed encode encode-parity decode; do
  timeout -k 10 120 python tools/bench_e2e.py --api capi --mode $m > $O/c5_$m.log 2>&1
done
for m in encode encode-parity decode; do
  timeout -k 10 120 python tools/bench_e2e.py --api capi --mode $m --k 29 --n 80 --ess 256 > $O/rs29_$m.log 2>&1
done
echo done
