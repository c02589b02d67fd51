#!/bin/bash
set -o pipefail
export PYTHONUNBUFFERED=1
for cfg in "1 16" "1 50" "1 100" "2 50"; do
  set -- $cfg
  timeout -k 10 120 python scripts/debug_r18_grads.py --quiet --groups $1 --batch $2 2>&1 | grep -v amdgpu.ids | tail -4 || exit 1
done
