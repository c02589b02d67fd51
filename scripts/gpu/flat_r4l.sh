#!/bin/bash
# stride-1 1x1 convs re-shaped onto 128-pixel rows (FLAT1X1): numerics, then ResNet-50 fp32 A/B
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_fp32_gpu.py tests/test_x6h_gpu.py > gpurun_out/flat_tests.log 2>&1; rc=$?; tail -1 gpurun_out/flat_tests.log
case $rc in 0) ;; *) grep -E "Error|assert|FAIL" gpurun_out/flat_tests.log | head -12; exit 1;; esac
run() { timeout -k 10 300 python -u benchmarks/bench_resnet50_dp.py --batch 256 --steps 5 --warmup 2 "$@" 2>&1 | grep '^{' | cut -c1-160; }
for F in 1 0 1 0; do echo "flat=$F $(DDL_F32_FLAT1X1=$F run)" || exit 1; done
