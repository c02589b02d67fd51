#!/bin/bash
# fp32 WGRAD on a side stream (DDL_WGRAD_OVERLAP=1) vs serial: fp32 tests with overlap, benches at 8 and 1 clients.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
DDL_WGRAD_OVERLAP=1 timeout -k 10 600 python -u -m pytest tests/test_fp32_gpu.py -q -x --timeout 300 --timeout-method thread > gpurun_out/ov_tests.log 2>&1 || { tail -30 gpurun_out/ov_tests.log; exit 1; }
tail -1 gpurun_out/ov_tests.log
for C in 1 8; do for O in 0 1; do
  T=$((6250 * C))
  DDL_WGRAD_OVERLAP=$O timeout -k 10 300 python -u bench.py --steps 3 --clients $C --train-size $T > gpurun_out/ov_bench_${C}_$O.log 2>&1 || { tail -20 gpurun_out/ov_bench_${C}_$O.log; exit 1; }
  echo "clients=$C overlap=$O $(tail -1 gpurun_out/ov_bench_${C}_$O.log | cut -c1-150)"
done; done
