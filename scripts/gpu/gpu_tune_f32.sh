#!/bin/bash
# X6 default: tune G=4,2,1; headline + per-client-count benches for both engines; X6 profile.
set -o pipefail
mkdir -p gpurun_out/prof_x6
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u scripts/conv_f32_tune.py --math x6 --out gpurun_out/f32_plans_x6_g421.json --groups 4 2 1 --budget-s 500 \
  > gpurun_out/r3i_tune.log 2>&1 || { tail -5 gpurun_out/r3i_tune.log; exit 1; }
tail -1 gpurun_out/r3i_tune.log
python - <<'PY'
import json
p='ddl25spring_amd/ops/f32_plans.json'
cur=json.load(open(p)); new=json.load(open('gpurun_out/f32_plans_x6_g421.json'))
cur['plans'].update(new['plans']); json.dump(cur,open(p,'w'),indent=1)
PY
for M in x6 mfma32; do
  for C in 8 4 2 1; do
    T=$((6250 * C))
    DDL_F32_MATH=$M timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --clients $C --train-size $T >> gpurun_out/r3i_bench.jsonl 2> gpurun_out/r3i_bench_$M$C.err || { tail -20 gpurun_out/r3i_bench_$M$C.err; exit 1; }
    tail -1 gpurun_out/r3i_bench.jsonl | cut -c1-200
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_x6 -o run -- python -u bench.py --steps 3 --warmup 1 \
  > gpurun_out/r3i_prof.log 2>&1 || { tail -20 gpurun_out/r3i_prof.log; exit 1; }
db=$(ls gpurun_out/prof_x6/*/run_results.db gpurun_out/prof_x6/run_results.db 2>/dev/null | head -n 1 || true)
[ -n "$db" ] && python scripts/prof_summary.py "$db" --top 40 > gpurun_out/r3i_prof_summary.txt
head -20 gpurun_out/r3i_prof_summary.txt
