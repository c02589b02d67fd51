#!/bin/bash
# graph-timed re-tune of the old-engine launches at 8 clients; A/B headline on the old vs merged table
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u scripts/conv_f32_tune.py --model resnet18 --math auto --groups 8 --skip-halo --budget-s 520 --out gpurun_out/r18_g8_plans.json > gpurun_out/r5t8_tune.log 2>&1 || { tail -5 gpurun_out/r5t8_tune.log; exit 1; }
tail -2 gpurun_out/r5t8_tune.log
cp ddl25spring_amd/ops/f32_plans.json gpurun_out/f32_plans_before_t8.json
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/r5t8_b.log 2>&1 || exit 1
echo "old  $(tail -1 gpurun_out/r5t8_b.log | cut -c95-160)"
python scripts/merge_plans.py gpurun_out/r18_g8_plans.json && cp ddl25spring_amd/ops/f32_plans.json gpurun_out/f32_plans_t8.json
for r in 1 2; do
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/r5t8_b.log 2>&1 || exit 1
echo "new  $(tail -1 gpurun_out/r5t8_b.log | cut -c95-160)"
cp gpurun_out/f32_plans_before_t8.json ddl25spring_amd/ops/f32_plans.json
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/r5t8_b.log 2>&1 || exit 1
echo "old  $(tail -1 gpurun_out/r5t8_b.log | cut -c95-160)"
cp gpurun_out/f32_plans_t8.json ddl25spring_amd/ops/f32_plans.json
done
