#!/bin/bash
# builds (here) or runs (GPU box: `gcm_var.sh run`) the AES-GCM T-table variants
D=$(dirname "$0")
# variants: copies (T-table layout) and exp (1 = no GHASH multiplies, 2 = no AES)
V=${V:-"0:0 32:0 64:0 32:1 32:2"}
TB=${TB:-1}
LIN=${LIN:-1}
WPC=${WPC:-1}
if [ "$1" = run ]; then
  for v in $V; do timeout -k 5 60 $D/gcm_var_${v/:/_}_t${TB}_l${LIN}_w$WPC || exit 1; done
else
  for v in $V; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++20 -x hip -DUPLINK_GCM_COPIES=${v%:*} -DUPLINK_GCM_EXP=${v#*:} -DUPLINK_GCM_TABLES=$TB -DUPLINK_GCM_LIN=$LIN -DUPLINK_GCM_WGS_PER_CU=$WPC \
      $D/gcm_var.cpp -o $D/gcm_var_${v/:/_}_t${TB}_l${LIN}_w$WPC || exit 1
  done
fi
