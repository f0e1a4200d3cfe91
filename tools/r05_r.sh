#!/bin/bash
# Round-5 call: waves per workgroup of the share-set pass for segments of at
# most 16 rows (UPLINK_EC_SETS_SMALL_WAVES 2 / 3 / 4): the one-set leg (m = 15)
# of the share-set bench, interleaved.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05/r}
mkdir -p $O
for r in 1 2; do
  for w in 2 3 4; do
    UPLINK_EC_SETS_SMALL_WAVES=$w timeout -k 10 200 python -u tools/bench_sets.py --reps 16 >> $O/bench_sets_small$w.json 2>> $O/err.log
  done
done
echo all-done > $O/done
