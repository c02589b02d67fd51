#!/bin/bash
# halo DGRAD with / without the BN-backward operand transform (and its write-out), per layer
set -o pipefail
export PYTHONUNBUFFERED=1
for L in c64 c128 c256; do for D in 0 1 2; do
  timeout -k 10 60 python scripts/conv_f32_bench.py --math auto --mode dgrad --layer $L --dybn $D --reps 20 2>&1 | tail -1 || exit 1
done; done
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_multirank_gpu.py -k fp32_resnet18 -s > gpurun_out/mr.log 2>&1; grep -E "fp32 ResNet|passed|failed" gpurun_out/mr.log | tail -2
