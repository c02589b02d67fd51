#!/bin/bash
# ResNet-50 DP (batch 256): bench + per-launch trace of one step.
set -o pipefail
tag=${1:-r50}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python benchmarks/bench_resnet50_dp.py --steps 10 --warmup 3 > $out/bench.log 2>&1 || { tail -5 $out/bench.log; exit 1; }
grep '^{' $out/bench.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/tr -o run -- python benchmarks/bench_resnet50_dp.py --steps 3 --warmup 2 > $out/tr.log 2>&1 || { tail -5 $out/tr.log; exit 1; }
f=$(ls $out/tr/*/run_kernel_trace.csv 2>/dev/null || ls $out/tr/run_kernel_trace.csv)
python scripts/step_trace.py $f > $out/step.txt
awk '{split($0,a,"  "); } {print}' /dev/null
rm -f $f
tail -n 1 $out/step.txt
