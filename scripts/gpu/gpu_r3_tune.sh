#!/bin/bash
# fp32 conv: numerics tests + plan tuning (per-layer TF/s) on one MI355X.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_fp32_gpu.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r3_fp32_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r3_fp32_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u scripts/conv_f32_tune.py --out gpurun_out/f32_plans_${TAG:-x}.json --groups ${GROUPS_:-8} --budget-s 420 \
  > gpurun_out/r3_tune_${TAG:-x}.log 2>&1
tail -2 gpurun_out/r3_tune_${TAG:-x}.log
