#!/bin/bash
# ResNet-50 fp32 plans: graph-timed halo sweep (3x3 s1, padded rows) + old-engine re-tune at batch 256,
# A/B on the ResNet-50 DP bench, ResNet-50 GPU tests on the merged table
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
echo "before $(timeout -k 10 400 python -u benchmarks/bench_resnet50_dp.py --steps 6 --warmup 3 2>&1 | tail -1 | cut -c70-150)" || exit 1
timeout -k 10 400 python -u scripts/halo_plan_probe.py --model resnet50 --G 1 --N 256 --reps 5 --out gpurun_out/r50_x6h_plans.json > gpurun_out/r5r50_probe.txt 2>&1 || { tail -5 gpurun_out/r5r50_probe.txt; exit 1; }
cut -c1-150 gpurun_out/r5r50_probe.txt
timeout -k 10 700 python -u scripts/conv_f32_tune.py --model resnet50 --groups 1 --batch 256 --math auto --skip-halo --budget-s 600 --out gpurun_out/r50_plans.json > gpurun_out/r5r50_tune.log 2>&1 || { tail -5 gpurun_out/r5r50_tune.log; exit 1; }
tail -2 gpurun_out/r5r50_tune.log | cut -c1-200
cp ddl25spring_amd/ops/f32_plans.json gpurun_out/f32_plans_before_r50.json
python scripts/merge_plans.py gpurun_out/r50_x6h_plans.json && python scripts/merge_plans.py gpurun_out/r50_plans.json && cp ddl25spring_amd/ops/f32_plans.json gpurun_out/f32_plans_r50.json
for r in 1 2; do
echo "after $(timeout -k 10 400 python -u benchmarks/bench_resnet50_dp.py --steps 6 --warmup 3 2>&1 | tail -1 | cut -c70-150)" || exit 1
done
