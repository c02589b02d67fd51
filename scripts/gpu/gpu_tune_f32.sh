#!/bin/bash
# Re-tune the fp32 conv plans (MATH=auto: both engines per layer; or x6 / mfma32) for G = 8, 4, 2, 1 clients (splits up to 128 at G <= 2), merge
# them into ddl25spring_amd/ops/f32_plans.json, then bench 8 and 1 clients with the new plans.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u scripts/conv_f32_tune.py --math ${MATH:-auto} --out gpurun_out/f32_plans_tuned.json --groups 8 4 2 1 --budget-s 900 \
  > gpurun_out/tune_all.log 2>&1 || { tail -5 gpurun_out/tune_all.log; exit 1; }
tail -1 gpurun_out/tune_all.log
python - <<'PY'
import json
p='ddl25spring_amd/ops/f32_plans.json'
cur=json.load(open(p)); new=json.load(open('gpurun_out/f32_plans_tuned.json'))
cur['plans'].update(new['plans']); json.dump(cur,open(p,'w'),indent=1)
json.dump(cur,open('gpurun_out/f32_plans_merged.json','w'),indent=1)
print("merged", len(new['plans']))
PY
for C in 8 1; do
  T=$((6250 * C))
  timeout -k 10 300 python -u bench.py --steps 3 --clients $C --train-size $T > gpurun_out/tune_bench_$C.log 2>&1 || { tail -20 gpurun_out/tune_bench_$C.log; exit 1; }
  echo "clients=$C $(tail -1 gpurun_out/tune_bench_$C.log | cut -c1-150)"
done
timeout -k 10 600 python -u -m pytest tests/test_fp32_gpu.py -q -x --timeout 300 --timeout-method thread > gpurun_out/tune_tests.log 2>&1 || { tail -30 gpurun_out/tune_tests.log; exit 1; }
tail -1 gpurun_out/tune_tests.log
