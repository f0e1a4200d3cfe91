#!/bin/bash
# Round-5 call: share-set launches on 3 (product) or 4 waves per workgroup
# (UPLINK_EC_SETS_MIN_WAVES), interleaved.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05/q}
mkdir -p $O
for r in 1 2; do
  timeout -k 10 200 python -u tools/bench_sets.py --reps 16 >> $O/bench_sets_w3.json 2>> $O/err.log
  UPLINK_EC_SETS_MIN_WAVES=4 timeout -k 10 200 python -u tools/bench_sets.py --reps 16 >> $O/bench_sets_w4.json 2>> $O/err.log
done
echo all-done > $O/done
