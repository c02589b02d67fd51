#!/bin/bash
# measured halo plans: sweep -> merge on the box -> tests + 1/2/4/8-client benches on the merged table
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/halo_plan_probe.py --G 1 2 4 8 --out gpurun_out/x6h_plans.json > gpurun_out/r5hp_probe.txt 2>&1 || { tail -5 gpurun_out/r5hp_probe.txt; exit 1; }
python scripts/merge_plans.py gpurun_out/x6h_plans.json && cp ddl25spring_amd/ops/f32_plans.json gpurun_out/f32_plans_hp.json
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_x6h_gpu.py tests/test_fp32_gpu.py > gpurun_out/r5hp_t.log 2>&1; rc=$?
tail -1 gpurun_out/r5hp_t.log; [ $rc = 0 ] || { grep -m5 "Error\|FAILED\|assert" gpurun_out/r5hp_t.log; exit 1; }
for C in 1 2 4 8; do
  timeout -k 10 300 python -u bench.py --clients $C --train-size $((6250 * C)) --steps 5 --warmup 2 > gpurun_out/r5hp_b.log 2>&1 || { tail -5 gpurun_out/r5hp_b.log; exit 1; }
  echo "clients=$C $(tail -1 gpurun_out/r5hp_b.log | cut -c100-200)"
done
