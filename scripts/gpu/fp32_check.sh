#!/bin/bash
# fp32 GPU tests (incl. the ResNet-50 step vs float64 / torch fp32) + headline bench at 8 and 1 clients.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_fp32_gpu.py -q -x --timeout 500 --timeout-method thread > gpurun_out/fc_tests.log 2>&1
rc=$?
tail -25 gpurun_out/fc_tests.log | grep -v "^$" | cut -c1-600
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for C in 8 1; do
  T=$((6250 * C))
  timeout -k 10 300 python -u bench.py --steps 3 --clients $C --train-size $T > gpurun_out/fc_bench_$C.log 2>&1 || { tail -20 gpurun_out/fc_bench_$C.log; exit 1; }
  echo "clients=$C $(tail -1 gpurun_out/fc_bench_$C.log | cut -c1-150)"
done
exit $rc
