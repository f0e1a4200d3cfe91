set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03/enc_q1
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_parity.log 2>&1
bash tools/exp/ab_bench.sh $O uplink_amd/lib/exp_base/libuplink_ec.so uplink_amd/lib/libuplink_ec.so
