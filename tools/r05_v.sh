#!/bin/bash
# Round-5 call: the share-set tests.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05/v}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_sets.py -m gpu > $O/pytest.log 2>&1
echo all-done > $O/done
