#!/bin/bash
# ResNet-50 at the reference's precision: the fp32 GPU tests (incl. the whole-network ResNet-50 step), then the DP bench in fp32 and bf16.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_fp32_gpu.py -q -x -k resnet50 --timeout 500 --timeout-method thread > gpurun_out/r50_test.log 2>&1 || { tail -30 gpurun_out/r50_test.log; exit 1; }
tail -1 gpurun_out/r50_test.log
for P in fp32 bf16; do
  timeout -k 10 400 python -u benchmarks/bench_resnet50_dp.py --precision $P --steps 8 --warmup 3 > gpurun_out/r50_$P.log 2>&1 || { tail -20 gpurun_out/r50_$P.log; exit 1; }
  tail -1 gpurun_out/r50_$P.log | cut -c1-250
done
