set -e
mkdir -p gpurun_out/r3gcm
for v in product gcmu2 gcmu4 product; do
  if [ $v = product ]; then L=uplink_amd/lib/libuplink_ec.so; else L=tools/exp/bin/var_$v/libuplink_ec.so; fi
  timeout -k 10 120 python -u -c "
import sys, runpy
sys.argv=['bench_gcm.py','--cpu-sample-s','0.5']
from uplink_amd import _native
_native.load('$L')
runpy.run_path('tools/bench_gcm.py', run_name='__main__')" > gpurun_out/r3gcm/$v.log 2>&1
  echo "$v: $(tail -1 gpurun_out/r3gcm/$v.log | cut -c1-300)" >> gpurun_out/r3gcm/summary.log
done
