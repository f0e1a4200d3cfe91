#!/bin/bash
# bench.py at several segments-per-launch on one box:  bash tools/exp/ab_batch.sh OUTDIR B1 B2 ...
set -e
O=$1; shift
mkdir -p $O
for i in 1 2; do
  for B in "$@"; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-other-configs --batch $B > $O/b${B}_$i.log 2>&1
  done
done
echo done
