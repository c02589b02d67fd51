#!/bin/bash
# LM-head DGRAD on the vendor GEMM (table entry) vs native, fp32 LLaMA bench A/B
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for V in base headv base headv; do
  cp gpurun_out/f32_plans_$V.json ddl25spring_amd/ops/f32_plans.json
  echo "$V $(timeout -k 10 300 python -u benchmarks/bench_llm.py --precision fp32 --steps 10 --warmup 3 2>&1 | tail -1 | cut -c50-100)" || exit 1
done
