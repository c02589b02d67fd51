#!/bin/bash
# conv_x6h 2-step chains: numerics (x6h + fp32 suites), per-layer FWD / DGRAD, headline
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_x6h_gpu.py tests/test_fp32_gpu.py > gpurun_out/x6c_tests.log 2>&1; rc=$?; tail -1 gpurun_out/x6c_tests.log
case $rc in 0) ;; *) grep -E "Error|assert|err |FAIL" gpurun_out/x6c_tests.log | head -12; exit 1;; esac
for M in fwd dgrad; do for L in c64 c128 c256; do
  timeout -k 10 60 python scripts/conv_f32_bench.py --math auto --mode $M --layer $L --reps 20 2>&1 | tail -1 || exit 1
done; done
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_x6c.json 2> gpurun_out/bench_x6c.err || exit 1
tail -1 gpurun_out/bench_x6c.json | cut -c1-200
