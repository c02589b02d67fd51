#!/bin/bash
# WGRAD side stream without record_stream: graph-pool memory, fp32 tests (incl. determinism), benches.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for C in 8 1; do
  timeout -k 10 300 python -u scripts/mem_probe.py $C > gpurun_out/om_mem_$C.log 2>&1 || { tail -5 gpurun_out/om_mem_$C.log; exit 1; }
  tail -1 gpurun_out/om_mem_$C.log
done
timeout -k 10 600 python -u -m pytest tests/test_fp32_gpu.py tests/test_overlap_gpu.py -q -x --timeout 500 --timeout-method thread > gpurun_out/om_tests.log 2>&1 || { tail -30 gpurun_out/om_tests.log; exit 1; }
tail -1 gpurun_out/om_tests.log
for C in 8 1; do
  T=$((6250 * C))
  timeout -k 10 300 python -u bench.py --steps 3 --clients $C --train-size $T > gpurun_out/om_bench_$C.log 2>&1 || { tail -20 gpurun_out/om_bench_$C.log; exit 1; }
  echo "clients=$C $(tail -1 gpurun_out/om_bench_$C.log | cut -c1-140)"
done
