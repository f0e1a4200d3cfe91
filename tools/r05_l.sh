#!/bin/bash
# Round-5 call: GHASH's Horner step on H^64's 8-bit table -- the GCM parity
# tests, then seal/open against the 4-bit table and with 16 / 24 T-table
# copies (variant libraries), interleaved.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05/l}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_aesgcm.py -m gpu > $O/pytest.log 2>&1
for r in 1 2; do
  UPLINK_GCM_GHASH8=0 timeout -k 10 120 python -u tools/bench_gcm.py --cpu-sample-s 1 >> $O/gcm_g4.json 2>> $O/gcm.err
  timeout -k 10 120 python -u tools/bench_gcm.py --cpu-sample-s 1 >> $O/gcm_g8.json 2>> $O/gcm.err
  timeout -k 10 120 python -u tools/bench_gcm.py --cpu-sample-s 1 --lib tools/exp/bin/var_c16/libuplink_ec.so >> $O/gcm_g8_c16.json 2>> $O/gcm.err
  timeout -k 10 120 python -u tools/bench_gcm.py --cpu-sample-s 1 --lib tools/exp/bin/var_c24/libuplink_ec.so >> $O/gcm_g8_c24.json 2>> $O/gcm.err
done
echo all-done > $O/done
