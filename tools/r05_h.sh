#!/bin/bash
# Round-5 call: the share-set and upload tests, the share-set bench (staging A/B),
# the decode wave-split A/B, and the
# share-set bench under rocprofv3 --kernel-trace --stats (per-kernel times of
# the prep and rebuild launches).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05/h}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_sets.py tests/test_segment.py tests/test_blake3.py -m gpu > $O/pytest.log 2>&1
timeout -k 10 200 python -u tools/bench_sets.py > $O/bench_sets.json 2> $O/bench_sets.err
UPLINK_EC_SETS_STAGE_DMA=1 timeout -k 10 200 python -u tools/bench_sets.py > $O/bench_sets_dma.json 2>> $O/bench_sets.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/bench_sets.py > $O/bench_sets_rocprof.log 2>&1
for rw in 4 5 6 8; do UPLINK_SL_WIDE_ROWS_PER_WAVE=$rw timeout -k 10 200 python -u tools/exp/ab_decode_rows.py >> $O/ab_decode_rows.json 2>> $O/ab_decode_rows.err; done
echo all-done > $O/done
