#!/bin/bash
# Per-launch kernel trace of one training step at 1 and 8 clients per GPU (csv kernel trace).
#   gpurun --timeout 600 -- bash scripts/gpu/gpu_trace1.sh <tag>
set -o pipefail
export TMPDIR=/tmp
tag=${1:-t}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/c1 -o run -- python bench.py --clients 1 --train-size 6250 --steps 2 --warmup 1 > $out/c1.log 2>&1 || exit 1
f=$(ls $out/c1/*/run_kernel_trace.csv 2>/dev/null || ls $out/c1/run_kernel_trace.csv)
python scripts/step_trace.py $f > $out/step_c1.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/c8 -o run -- python bench.py --steps 2 --warmup 1 > $out/c8.log 2>&1 || exit 1
f=$(ls $out/c8/*/run_kernel_trace.csv 2>/dev/null || ls $out/c8/run_kernel_trace.csv)
python scripts/step_trace.py $f > $out/step_c8.txt
rm -f $out/c1/*/run_kernel_trace.csv $out/c8/*/run_kernel_trace.csv $out/c1/run_kernel_trace.csv $out/c8/run_kernel_trace.csv
tail -n 1 $out/step_c1.txt $out/step_c8.txt
