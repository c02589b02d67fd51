#!/bin/bash
# Standalone builds of csrc/kernels/mlp_epoch.hip with compile-time variants, for A/B timing on the
# GPU box through DDL_MLP_LIB (ops/mlp_epoch.py). Usage: bash scripts/mlp_epoch_variants.sh NAME "-DFLAG=V ..." ...
set -e
cd "$(dirname "$0")/.."
mkdir -p ddl25spring_amd/lib/variants
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Icsrc/include $flags \
    csrc/kernels/mlp_epoch.hip -o ddl25spring_amd/lib/variants/mlp_$name.so
  echo "built mlp_$name.so ($flags)"
done
