#!/bin/bash
# ResNet-50 DP: flattened stride-1 1x1 convs (halo kernels) per mode subset, A/B against the default
set -o pipefail
mkdir -p gpurun_out
for F in 0 w d f fd dw 0; do
  DDL_F32_FLAT1X1=$F timeout -k 10 300 python -u benchmarks/bench_resnet50_dp.py --steps 6 --warmup 3 > gpurun_out/flat_$F.log 2>&1 || { tail -5 gpurun_out/flat_$F.log; exit 1; }
  echo "flat=$F $(grep '^{' gpurun_out/flat_$F.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
