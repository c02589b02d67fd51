#!/bin/bash
# graph-timed re-tune of the fp32 LLaMA linears (native plans + vendor GEMM), A/B on the LLM bench
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
echo "before $(timeout -k 10 300 python -u benchmarks/bench_llm.py --precision fp32 --steps 10 --warmup 3 2>&1 | tail -1 | cut -c50-130)" || exit 1
cp ddl25spring_amd/ops/f32_plans.json gpurun_out/f32_plans_before_l2.json
timeout -k 10 600 python -u scripts/conv_f32_tune.py --model llama288 --math auto --budget-s 500 --out gpurun_out/llm_plans2.json > gpurun_out/llm_tune2.log 2>&1 || { tail -20 gpurun_out/llm_tune2.log; exit 1; }
python scripts/merge_plans.py gpurun_out/llm_plans2.json && cp ddl25spring_amd/ops/f32_plans.json gpurun_out/f32_plans_l2.json
grep -c '"blas:' gpurun_out/llm_plans2.json
for r in 1 2; do
echo "after $(timeout -k 10 300 python -u benchmarks/bench_llm.py --precision fp32 --steps 10 --warmup 3 2>&1 | tail -1 | cut -c50-130)" || exit 1
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_llama_f32_gpu.py > gpurun_out/r5l2_t.log 2>&1; rc=$?
tail -1 gpurun_out/r5l2_t.log; [ $rc = 0 ] || { grep -m5 "Error\|FAILED\|assert" gpurun_out/r5l2_t.log; exit 1; }
