#!/bin/bash
# Round-5 measurement call (GPU box): the GPU suite, the share-set and upload
# benches, the bench line; then, last (a timed-out step ends the call), the
# checked C client with a cold and a warm run-time-compile cache and the
# library's log on, to show what process exit waits for.
set -e
O=gpurun_out/${1:-r05/d}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1
timeout -k 10 200 python -u tools/bench_sets.py > $O/bench_sets.json 2> $O/bench_sets.err
UPLINK_EC_SETS_MERGE=1 timeout -k 10 200 python -u tools/bench_sets.py > $O/bench_sets_merge.json 2> $O/bench_sets_merge.err
timeout -k 10 200 python -u tools/bench_segment.py > $O/bench_segment.log 2>&1
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1
# evidence for the checked-client timeout: a ticker keeps output flowing while a compile runs
( while sleep 20; do date +%T >> $O/ticker.log; done ) &
T=$!
export UPLINK_EC_LOG=1
rc=0
( time UPLINK_EC_JIT_CACHE=$PWD/$O/jit timeout -k 10 170 tests/c/build/abi_test_checked ) > $O/abi_checked_cold.log 2>&1 || rc=$?
echo "exit $rc" >> $O/abi_checked_cold.log
if [ $rc -eq 0 ]; then  # (nothing more on the GPU after a time limit)
  ( time UPLINK_EC_JIT_CACHE=$PWD/$O/jit timeout -k 10 170 tests/c/build/abi_test_checked ) > $O/abi_checked_warm.log 2>&1 || true
fi
kill $T
echo all-done > $O/done
