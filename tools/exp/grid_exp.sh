set -e
mkdir -p gpurun_out/s9
for M in 1 2 4 1000; do
  UPLINK_EXP_GRID_MULT=$M timeout -k 10 200 python bench.py --no-cpu-baseline --no-other-configs --steps 5 > gpurun_out/s9/bench_m$M.log 2>&1
done
echo done
