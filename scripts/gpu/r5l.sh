#!/bin/bash
# tune the fp32 LLaMA-288d linears (native engines + vendor fp32 GEMM), merge the table on the box,
# then the fp32 LLM bench and LLaMA fp32 tests on the merged table
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
echo "before $(timeout -k 10 300 python -u benchmarks/bench_llm.py --precision fp32 --steps 10 --warmup 3 2>&1 | tail -1 | cut -c1-150)" || exit 1
timeout -k 10 600 python -u scripts/conv_f32_tune.py --model llama288 --math auto --budget-s 500 --out gpurun_out/llm_plans.json > gpurun_out/llm_tune.log 2>&1 || { tail -20 gpurun_out/llm_tune.log; exit 1; }
python scripts/merge_plans.py gpurun_out/llm_plans.json && cp ddl25spring_amd/ops/f32_plans.json gpurun_out/f32_plans_merged.json
grep -c blas gpurun_out/llm_plans.json
echo "after $(timeout -k 10 300 python -u benchmarks/bench_llm.py --precision fp32 --steps 10 --warmup 3 2>&1 | tail -1 | cut -c1-150)" || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_llama_f32_gpu.py > gpurun_out/r5l_t.log 2>&1; rc=$?
tail -1 gpurun_out/r5l_t.log; [ $rc = 0 ] || { grep -m5 "Error\|FAILED\|assert" gpurun_out/r5l_t.log; exit 1; }
