#!/bin/bash
set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_fp32_gpu.py > gpurun_out/ws1_tests.log 2>&1; rc=$?; tail -1 gpurun_out/ws1_tests.log
case $rc in 0) ;; *) grep -E "Error|assert" gpurun_out/ws1_tests.log | head -5; exit 1;; esac
for L in c64 c128 c256 c512; do timeout -k 10 60 python scripts/conv_f32_bench.py --math auto --mode wgrad --layer $L --reps 20 2>&1 | tail -1 || exit 1; done
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 2>&1 | grep '^{' | cut -c1-200 || exit 1
timeout -k 10 300 python -u bench.py --clients 1 --train-size 6250 --steps 5 --warmup 2 2>&1 | grep '^{' | cut -c1-200 || exit 1
