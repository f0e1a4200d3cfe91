#!/bin/bash
# Round-5 call: the share-set bench (with its Decode leg).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05/w}
mkdir -p $O
timeout -k 10 200 python -u tools/bench_sets.py > $O/bench_sets.json 2> $O/err.log
echo all-done > $O/done
