#!/bin/bash
# VFL/tabular on the fused optimizer; re-tune fp32 conv plans for G=4,2,1; reference eager (3 rounds).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_tabular_gpu.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r3e_tab.log 2>&1 || { tail -30 gpurun_out/r3e_tab.log; exit 1; }
tail -2 gpurun_out/r3e_tab.log
timeout -k 10 600 python -u scripts/conv_f32_tune.py --out gpurun_out/f32_plans_g421.json --groups 4 2 1 --budget-s 520 \
  > gpurun_out/r3e_tune.log 2>&1 || { tail -5 gpurun_out/r3e_tune.log; exit 1; }
tail -2 gpurun_out/r3e_tune.log
for v in faithful tuned_fp32; do
  timeout -k 10 400 python -u benchmarks/bench_reference_eager.py --variant $v --steps 3 --warmup 1 \
    >> gpurun_out/reference_eager_r3e.jsonl 2> gpurun_out/r3e_ref_$v.err || { tail -5 gpurun_out/r3e_ref_$v.err; exit 1; }
  tail -1 gpurun_out/reference_eager_r3e.jsonl
done
