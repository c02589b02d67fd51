#!/bin/bash
# halo WGRAD bring-up: LDS misaligned-read probe, numerics, layer timing (halo vs conv_f32), bench
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 5 30 ./scripts/lds_unaligned.bin || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_x6h_gpu.py -k x6hw > gpurun_out/hw_tests.log 2>&1; rc=$?; tail -3 gpurun_out/hw_tests.log
case $rc in 0) ;; *) grep -E "Error|assert|err " gpurun_out/hw_tests.log | head -8; exit 1;; esac
for L in c64 c128 c256; do for H in 1 0; do
  DDL_F32_HALO_WGRAD=$H timeout -k 10 60 python scripts/conv_f32_bench.py --math auto --mode wgrad --layer $L --reps 20 2>&1 | tail -1 | sed "s/^/hw=$H /" || exit 1
done; done
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_fp32_gpu.py > gpurun_out/hw_fp32.log 2>&1; tail -1 gpurun_out/hw_fp32.log
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 2>&1 | grep '^{' | cut -c1-220 || exit 1
timeout -k 10 300 python -u bench.py --clients 1 --train-size 6250 --steps 5 --warmup 2 2>&1 | grep '^{' | cut -c1-220 || exit 1
