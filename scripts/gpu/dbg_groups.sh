#!/bin/bash
# ResNet-18 fp32 step vs float64 at several (groups, batch, split-K target) settings.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for cfg in "1 50 0" "2 50 0" "1 16 0" "1 50 1" "2 50 1" "1 64 0" "1 100 0"; do
  set -- $cfg
  timeout -k 10 120 python scripts/debug_r18_grads.py --quiet --groups $1 --batch $2 --target-wg $3 2>&1 | tail -3 || exit 1
done
timeout -k 10 120 python scripts/debug_r18_grads.py --quiet --groups 1 --batch 50 --halo 0 2>&1 | tail -3 || exit 1
