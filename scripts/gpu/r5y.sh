#!/bin/bash
# BN fold unrolled final sum: BN tests + 1-client / 8-client bench; LLM token-row geometry A/B + llama tests
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fp32_gpu.py -k "bn" > gpurun_out/r5y_bn.log 2>&1; rc=$?
tail -1 gpurun_out/r5y_bn.log
[ $rc = 0 ] || { grep -m3 "Error\|FAILED" gpurun_out/r5y_bn.log; exit 1; }
for C in 1 8; do
  echo "clients=$C $(timeout -k 10 300 python -u bench.py --clients $C --steps 5 --warmup 2 2>&1 | tail -1 | cut -c1-110)" || exit 1
done
for R in 0 1; do
  echo "ROWS=$R $(DDL_F32_LLM_ROWS=$R timeout -k 10 300 python -u benchmarks/bench_llm.py --precision fp32 --steps 10 --warmup 3 2>&1 | tail -1 | cut -c1-160)" || exit 1
done
DDL_F32_LLM_ROWS=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_llama_f32_gpu.py > gpurun_out/r5y_llm.log 2>&1; rc=$?
tail -1 gpurun_out/r5y_llm.log
[ $rc = 0 ] || { grep -m3 "Error\|FAILED" gpurun_out/r5y_llm.log; exit 1; }
