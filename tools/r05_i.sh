#!/bin/bash
# Round-5 call: the share-set bench with the clock settled at the timed loop's
# duty cycle, twice (box variance), and the bench line.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05/i}
mkdir -p $O
timeout -k 10 200 python -u tools/bench_sets.py > $O/bench_sets.json 2> $O/bench_sets.err
timeout -k 10 200 python -u tools/bench_sets.py > $O/bench_sets2.json 2>> $O/bench_sets.err
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1
echo all-done > $O/done
