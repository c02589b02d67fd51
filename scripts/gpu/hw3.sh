#!/bin/bash
# halo WGRAD: tests, per-layer timing at 8 and 1 clients, then the headline with / without it
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_x6h_gpu.py -k x6hw > gpurun_out/hw_tests.log 2>&1; rc=$?; tail -1 gpurun_out/hw_tests.log
case $rc in 0) ;; *) grep -E "Error|assert|err " gpurun_out/hw_tests.log | head -8; exit 1;; esac
for G in 8 1; do for L in c64 c128; do for H in 1 0; do
  DDL_F32_HALO_WGRAD=$H timeout -k 10 60 python scripts/conv_f32_bench.py --math auto --mode wgrad --layer $L --G $G --reps 20 2>&1 | tail -1 | sed "s/^/hw=$H /" || exit 1
done; done; done
for H in 1 0; do
  DDL_F32_HALO_WGRAD=$H timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_hw$H.json 2> gpurun_out/bench_hw$H.err || exit 1
  echo "hw=$H $(tail -1 gpurun_out/bench_hw$H.json | cut -c1-200)"
done
