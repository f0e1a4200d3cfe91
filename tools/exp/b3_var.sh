#!/bin/bash
# builds (here) or runs (on the GPU box: `b3_var.sh run`) the b3_var variants
D=$(dirname "$0")
V="256:1 256:0 512:1 512:0 1024:1 1024:0 128:1"
if [ "$1" = run ]; then
  for v in $V; do timeout -k 5 60 $D/b3_var_${v/:/_} || exit 1; done
else
  for v in $V; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++20 -x hip -DUPLINK_B3_GROUP=${v%:*} -DUPLINK_B3_LINES=${v#*:} \
      $D/b3_var.cpp -o $D/b3_var_${v/:/_} || exit 1
  done
fi
