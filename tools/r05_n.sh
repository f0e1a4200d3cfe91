#!/bin/bash
# Round-5 call: AES-GCM grid size (workgroups per CU in the grid), interleaved.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05/n}
mkdir -p $O
for r in 1 2; do
  for g in 4 8 16 32; do
    UPLINK_GCM_GRID_PER_CU=$g timeout -k 10 120 python -u tools/bench_gcm.py --cpu-sample-s 1 >> $O/gcm_grid$g.json 2>> $O/gcm.err
  done
done
echo all-done > $O/done
