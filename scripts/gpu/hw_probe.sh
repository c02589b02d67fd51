#!/bin/bash
# halo WGRAD timing probes: which phase costs what (DDL_HW_PROBE bits: 1 no LDS staging, 2 no MFMA,
# 4 no loads, 8 no IEEE adds, 16 no shifted windows; results wrong)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 DDL_F32_HALO_WGRAD=1
for L in ${LAYERS:-c128 c256}; do for P in ${PROBES:-0 5 13 21 29 2}; do
  DDL_HW_PROBE=$P timeout -k 10 60 python scripts/conv_f32_bench.py --math auto --mode wgrad --layer $L --reps 20 2>&1 | tail -1 | sed "s/^/probe=$P /" || exit 1
done; done
