#!/bin/bash
# LLaMA-288d (dp1 pp1, batch 32): per-launch trace of one graph-replayed step.
set -o pipefail
tag=${1:-llm}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/tr -o run -- python benchmarks/bench_llm.py --steps 5 --warmup 3 > $out/tr.log 2>&1 || { tail -5 $out/tr.log; exit 1; }
grep '^{' $out/tr.log | cut -c1-200
f=$(ls $out/tr/*/run_kernel_trace.csv 2>/dev/null || ls $out/tr/run_kernel_trace.csv)
python scripts/step_trace.py $f adam_kernel > $out/step.txt
rm -f $f
tail -n 1 $out/step.txt
