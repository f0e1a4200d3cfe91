#!/bin/bash
# Round-5 call: AES-GCM with GHASH's 8-bit Horner table -- T-table copies
# (32 / 16 / 8) and a 128-VGPR budget (4 waves per SIMD), variant libraries,
# interleaved.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05/l3}
mkdir -p $O
for r in 1 2; do
  timeout -k 10 120 python -u tools/bench_gcm.py --cpu-sample-s 1 >> $O/gcm_c32.json 2>> $O/gcm.err
  for v in c16 c16w4 c8 c8w4; do
    timeout -k 10 120 python -u tools/bench_gcm.py --cpu-sample-s 1 --lib tools/exp/bin/var_$v/libuplink_ec.so >> $O/gcm_$v.json 2>> $O/gcm.err
  done
done
echo all-done > $O/done
