#!/bin/bash
# WGRAD split-K reduce with four interleaved partial sums: numerics + determinism, then benches
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_fp32_gpu.py tests/test_x6h_gpu.py tests/test_fl_gpu.py > gpurun_out/red_tests.log 2>&1; rc=$?; tail -1 gpurun_out/red_tests.log
case $rc in 0) ;; *) grep -E "Error|assert|FAIL" gpurun_out/red_tests.log | head -12; exit 1;; esac
val() { python3 -c "import json,sys; print(json.loads(sys.stdin.readlines()[-1])['value'])"; }
for C in 1 8; do
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --clients $C --train-size $((6250 * C)) > gpurun_out/red_c$C.json 2> gpurun_out/red_c$C.err || exit 1
  echo "clients=$C $(val < gpurun_out/red_c$C.json)"
done
