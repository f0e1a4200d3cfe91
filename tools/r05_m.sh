#!/bin/bash
# Round-5 call: AES-GCM product (8-bit Horner table, 16 T-table copies, four
# workgroups per CU): parity tests, the GCM bench, and the bench under
# rocprofv3 --kernel-trace --stats.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05/m2}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_aesgcm.py tests/test_pipeline.py -m gpu > $O/pytest.log 2>&1
timeout -k 10 200 python -u tools/bench_gcm.py > $O/bench_gcm.json 2> $O/bench_gcm.err
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/bench_gcm.py --cpu-sample-s 1 > $O/bench_gcm_rocprof.log 2>&1
echo all-done > $O/done
