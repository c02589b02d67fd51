#!/bin/bash
# graph-timed plan sweeps: halo FWD/DGRAD/WGRAD (probe) + old-engine launches at 1/2/4 clients (tuner),
# merged on the box, then tests and the clients-per-GPU benches on the merged table
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/halo_plan_probe.py --G 1 2 4 8 --out gpurun_out/x6h_plans2.json > gpurun_out/r5tu_probe.txt 2>&1 || { tail -5 gpurun_out/r5tu_probe.txt; exit 1; }
grep wgrad gpurun_out/r5tu_probe.txt | cut -c1-200
timeout -k 10 500 python -u scripts/conv_f32_tune.py --model resnet18 --math auto --groups 1 2 4 --skip-halo --budget-s 420 --out gpurun_out/r18_g124_plans.json > gpurun_out/r5tu_tune.log 2>&1 || { tail -5 gpurun_out/r5tu_tune.log; exit 1; }
tail -2 gpurun_out/r5tu_tune.log
python scripts/merge_plans.py gpurun_out/x6h_plans2.json && python scripts/merge_plans.py gpurun_out/r18_g124_plans.json && cp ddl25spring_amd/ops/f32_plans.json gpurun_out/f32_plans_tu.json
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_x6h_gpu.py tests/test_fp32_gpu.py > gpurun_out/r5tu_t.log 2>&1; rc=$?
tail -1 gpurun_out/r5tu_t.log; [ $rc = 0 ] || { grep -m5 "Error\|FAILED\|assert" gpurun_out/r5tu_t.log; exit 1; }
for C in 1 2 4 8; do
  timeout -k 10 300 python -u bench.py --clients $C --train-size $((6250 * C)) --steps 5 --warmup 2 > gpurun_out/r5tu_b.log 2>&1 || { tail -5 gpurun_out/r5tu_b.log; exit 1; }
  echo "clients=$C $(tail -1 gpurun_out/r5tu_b.log | cut -c95-200)"
done
