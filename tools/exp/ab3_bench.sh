#!/bin/bash
# A/B/C of three library builds in the bench (GPU box), alternating:
#   bash tools/exp/ab3_bench.sh OUTDIR LIB_A LIB_B LIB_C [bench args]
set -e
O=$1; A=$2; B=$3; C=$4; shift 4
mkdir -p $O
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-other-configs --lib $A "$@" > $O/a$i.log 2>&1
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-other-configs --lib $B "$@" > $O/b$i.log 2>&1
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-other-configs --lib $C "$@" > $O/c$i.log 2>&1
done
echo done
