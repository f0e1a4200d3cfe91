#!/bin/bash
# Round-5 call: one-segment latency against the rebuild's prefetch depth
# (UPLINK_EC_REBUILD_DEPTH 1 / 2 / 3: chunks of LDS-DMA in flight ahead of the
# straight-line body), through the share-set bench's single-segment and
# batched-API legs.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05/p}
mkdir -p $O
for r in 1 2; do
  for d in 1 2 3; do
    UPLINK_EC_REBUILD_DEPTH=$d timeout -k 10 200 python -u tools/bench_sets.py --reps 12 >> $O/bench_sets_depth$d.json 2>> $O/err.log
  done
done
echo all-done > $O/done
