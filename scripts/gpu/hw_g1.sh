#!/bin/bash
# halo WGRAD vs conv_f32 WGRAD at 1 and 2 clients (split rule: up to 128 slices of >= 3 tiles)
set -o pipefail
export PYTHONUNBUFFERED=1
for G in 1 2; do for L in c64 c128; do for H in 1 0; do
  DDL_F32_HALO_WGRAD=$H timeout -k 10 60 python scripts/conv_f32_bench.py --math auto --mode wgrad --layer $L --G $G --reps 50 2>&1 | tail -1 | sed "s/^/hw=$H /" || exit 1
done; done; done
