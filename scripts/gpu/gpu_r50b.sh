#!/bin/bash
set -o pipefail
tag=${1:-r50b}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k prep > $out/t.log 2>&1 || { tail -20 $out/t.log; exit 1; }
tail -n 1 $out/t.log
for i in 1 2; do
timeout -k 10 300 python benchmarks/bench_resnet50_dp.py --steps 10 --warmup 3 > $out/bench$i.log 2>&1 || { tail -5 $out/bench$i.log; exit 1; }
grep '^{' $out/bench$i.log | cut -c1-200
done
