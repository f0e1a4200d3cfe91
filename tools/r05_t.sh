#!/bin/bash
# Round-5 call: fused Decode with its inputs interleaved (chosen shares among
# the others): the decode GPU tests, then Decode with detection k+1..k+20
# against number order (UPLINK_EC_DECODE_INTERLEAVE=0), interleaved.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05/t}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_sets.py -m gpu -k "decode or Decode or correct or sets" > $O/pytest.log 2>&1
for r in 1 2; do
  UPLINK_EC_DECODE_INTERLEAVE=0 timeout -k 10 150 python -u tools/exp/ab_decode_rows.py >> $O/ab_dec_sorted.json 2>> $O/ab_dec.err
  timeout -k 10 150 python -u tools/exp/ab_decode_rows.py >> $O/ab_dec_interleaved.json 2>> $O/ab_dec.err
done
echo all-done > $O/done
