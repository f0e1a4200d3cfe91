#!/bin/bash
# Round-5 call: Decode's fused pass with syndromes against infectious' chosen
# shares -- its GPU tests, the share-set tests (host mirror included), then
# Decode with detection k+1..k+20.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05/k}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_sets.py -m gpu -k "decode or sets or Decode or correct" > $O/pytest.log 2>&1
for r in 1 2; do
  timeout -k 10 150 python -u tools/exp/ab_decode_rows.py >> $O/ab_dec.json 2>> $O/ab_dec.err
done
echo all-done > $O/done
