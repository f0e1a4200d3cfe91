#!/bin/bash
# Round-5 call: one-segment share-set calls with the record in the prep
# launch's arguments: the share-set and decode tests, then the share-set bench
# twice (its single-segment leg).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05/u}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_sets.py tests/test_gpu_parity.py -m gpu -k "sets or decode or Decode or batched" > $O/pytest.log 2>&1
timeout -k 10 200 python -u tools/bench_sets.py > $O/bench_sets.json 2> $O/err.log
timeout -k 10 200 python -u tools/bench_sets.py > $O/bench_sets2.json 2>> $O/err.log
echo all-done > $O/done
