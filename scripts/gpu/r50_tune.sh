#!/bin/bash
# ResNet-50 (ImageNet 224, batch 256, 1 rank) fp32 conv plans: tune, merge, bench native fp32 vs stock torch fp32.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u scripts/conv_f32_tune.py --math auto --model resnet50 --out gpurun_out/f32_plans_r50.json --groups 1 --batch 256 --budget-s 780 \
  > gpurun_out/tune_r50.log 2>&1 || { tail -5 gpurun_out/tune_r50.log; exit 1; }
tail -1 gpurun_out/tune_r50.log
python - <<'PY'
import json
p='ddl25spring_amd/ops/f32_plans.json'
cur=json.load(open(p)); new=json.load(open('gpurun_out/f32_plans_r50.json'))
cur['plans'].update(new['plans']); json.dump(cur,open(p,'w'),indent=1)
json.dump(cur,open('gpurun_out/f32_plans_merged_r50.json','w'),indent=1)
print("merged", len(new['plans']))
PY
timeout -k 10 400 python -u benchmarks/bench_resnet50_dp.py --precision fp32 --steps 8 --warmup 3 > gpurun_out/r50_fp32_tuned.log 2>&1 || { tail -20 gpurun_out/r50_fp32_tuned.log; exit 1; }
tail -1 gpurun_out/r50_fp32_tuned.log | cut -c1-220
MIOPEN_FIND_MODE=FAST timeout -k 10 500 python -u benchmarks/bench_resnet50_torch.py --batch 256 --steps 8 --warmup 3 > gpurun_out/r50_torch.log 2>&1 || { tail -20 gpurun_out/r50_torch.log; exit 1; }
tail -1 gpurun_out/r50_torch.log | cut -c1-220
