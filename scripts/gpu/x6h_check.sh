#!/bin/bash
# Halo X6 kernel: numerics vs float64, per-layer timing halo on/off, one short headline bench.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T=${1:-x6h}
timeout -k 10 400 python -u -m pytest tests/test_x6h_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
for L in c64 c128 c256 c512; do for O in fwd dgrad; do for H in 0 1; do
  timeout -k 10 60 python scripts/conv_f32_bench.py --math auto --halo $H --mode $O --layer $L --reps 20 2>&1 | tail -1 >> gpurun_out/${T}_layers.log || { tail -5 gpurun_out/${T}_layers.log; exit 1; }
done; done; done
cat gpurun_out/${T}_layers.log
timeout -k 10 300 python -u bench.py --steps 3 --warmup 2 > gpurun_out/${T}_bench.log 2>&1 || { tail -30 gpurun_out/${T}_bench.log; exit 1; }
tail -1 gpurun_out/${T}_bench.log | cut -c1-400
