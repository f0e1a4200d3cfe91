#!/bin/bash
# builds (here) or runs (GPU box: `gcm_var.sh run`) the AES-GCM T-table variants
D=$(dirname "$0")
if [ "$1" = run ]; then
  for c in 0 32 64; do timeout -k 5 60 $D/gcm_var_$c || exit 1; done
else
  for c in 0 32 64; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++20 -x hip -DUPLINK_GCM_COPIES=$c $D/gcm_var.cpp -o $D/gcm_var_$c || exit 1
  done
fi
