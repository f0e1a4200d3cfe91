#!/bin/bash
# Round-5 call: the smoke test (with its share-set call) and the share-set tests.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05/o}
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_sets.py -m gpu > $O/pytest.log 2>&1
echo all-done > $O/done
