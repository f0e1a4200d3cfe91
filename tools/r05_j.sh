#!/bin/bash
# Round-5 call: GCM with two slots per lane (parity tests, then A/B against one
# slot per lane, interleaved), the share-set tests, and the decode k+20 A/B of
# the wide-wave chunk size and prefetch depth (tools/exp/bin/var_w1: one input
# per wave per chunk).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05/j}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_aesgcm.py tests/test_sets.py -m gpu > $O/pytest.log 2>&1
for r in 1 2; do
  UPLINK_GCM_ILP=1 timeout -k 10 120 python -u tools/bench_gcm.py --cpu-sample-s 1 >> $O/gcm_ilp1.json 2>> $O/gcm.err
  timeout -k 10 120 python -u tools/bench_gcm.py --cpu-sample-s 1 >> $O/gcm_ilp2.json 2>> $O/gcm.err
done
for r in 1 2; do
  timeout -k 10 150 python -u tools/exp/ab_decode_rows.py 20 >> $O/ab_dec.json 2>> $O/ab_dec.err
  timeout -k 10 150 python -u tools/exp/ab_decode_rows.py --lib=tools/exp/bin/var_w1/libuplink_ec.so 20 >> $O/ab_dec.json 2>> $O/ab_dec.err
  UPLINK_EC_REBUILD_DEPTH=2 timeout -k 10 150 python -u tools/exp/ab_decode_rows.py --lib=tools/exp/bin/var_w1/libuplink_ec.so 20 >> $O/ab_dec.json 2>> $O/ab_dec.err
done
echo all-done > $O/done
