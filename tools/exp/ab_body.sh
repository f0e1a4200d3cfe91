#!/bin/bash
# A/B of bench.py --body auto vs straight-line on one box, alternating:
#   bash tools/exp/ab_body.sh OUTDIR [bench args]
set -e
O=$1; shift
mkdir -p $O
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-other-configs "$@" > $O/auto$i.log 2>&1
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-other-configs --body straight-line "$@" > $O/sl$i.log 2>&1
done
echo done
