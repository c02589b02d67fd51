#!/bin/bash
# X6 with store-time split: fp32 numerics (both engines), per-layer timing exact vs X6, X6 re-tune,
# headline bench X6, PMC of one layer.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_fp32_gpu.py -q --timeout 300 --timeout-method thread > gpurun_out/r3h_fp32.log 2>&1
rc=$?
tail -4 gpurun_out/r3h_fp32.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for L in c64 c128 c256 c512 c128s2 sc128; do for O in fwd dgrad wgrad; do for M in mfma32 x6; do
  timeout -k 10 60 python scripts/conv_f32_bench.py --math $M --mode $O --layer $L --reps 20 >> gpurun_out/r3h_layers.log 2>&1 || { tail -5 gpurun_out/r3h_layers.log; exit 1; }
done; done; done
cat gpurun_out/r3h_layers.log
timeout -k 10 500 python -u scripts/conv_f32_tune.py --math x6 --out gpurun_out/f32_plans_x6b_g8.json --groups 8 --budget-s 400 \
  > gpurun_out/r3h_tune_x6.log 2>&1 || { tail -5 gpurun_out/r3h_tune_x6.log; exit 1; }
tail -1 gpurun_out/r3h_tune_x6.log
cp gpurun_out/f32_plans_x6b_g8.json /tmp/x6plans.json
DDL_F32_MATH=x6 timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 > gpurun_out/r3h_bench_x6.log 2>&1 || { tail -20 gpurun_out/r3h_bench_x6.log; exit 1; }
tail -1 gpurun_out/r3h_bench_x6.log
timeout -k 10 600 bash scripts/gpu/pmc_f32.sh "mfma32 x6" "fwd" "c64" > gpurun_out/r3h_pmc.log 2>&1 || { tail -5 gpurun_out/r3h_pmc.log; exit 1; }
python scripts/pmc_waits_summary.py gpurun_out/pmcf convf32 > gpurun_out/r3h_pmc_summary.txt 2>&1
cat gpurun_out/r3h_pmc_summary.txt
