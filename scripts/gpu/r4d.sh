#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 5 60 ./scripts/mfma_rounding.bin | tee gpurun_out/mfma_rounding.txt || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_multirank_gpu.py -k fp32_resnet18 -s > gpurun_out/r4d_multirank.log 2>&1; rc=$?
grep -E "fp32 ResNet|passed|failed" gpurun_out/r4d_multirank.log | tail -3
case $rc in 124|134|137|139) exit $rc;; esac
exit 0
