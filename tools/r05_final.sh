#!/bin/bash
# Round-5 final measurement set (GPU box): the GPU suite, the smoke test, the
# round's measurement script (bench line, bench under rocprofv3 --kernel-trace
# --stats, FETCH_SIZE / WRITE_SIZE and SQ passes), the share-set and upload
# benches.  Each GPU step has its own time limit; the first failure ends it.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05/final}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
bash tools/prof_round.sh ${1:-r05/final}
timeout -k 10 200 python -u tools/bench_sets.py > $O/bench_sets.json 2> $O/bench_sets.err
timeout -k 10 200 python -u tools/bench_segment.py > $O/bench_segment.log 2>&1
echo all-done > $O/done
