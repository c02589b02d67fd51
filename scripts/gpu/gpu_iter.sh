#!/bin/bash
# Generic iteration: all GPU tests, then the headline bench at 8 and 1 clients (+ ResNet-50 DP
# with ITER_R50=1). Every step is time-limited and the script stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tg.log 2>&1 || { tail -30 gpurun_out/tg.log; exit 1; }
tail -2 gpurun_out/tg.log
timeout -k 10 200 python bench.py --steps 3 --warmup 1 > gpurun_out/hb8.log 2>&1 || { tail -20 gpurun_out/hb8.log; exit 1; }
grep '^{' gpurun_out/hb8.log | cut -c1-200
timeout -k 10 200 python bench.py --clients 1 --train-size 6250 --steps 3 --warmup 1 > gpurun_out/hb1.log 2>&1 || { tail -20 gpurun_out/hb1.log; exit 1; }
grep '^{' gpurun_out/hb1.log | cut -c1-200
if [ -n "$ITER_R50" ]; then
  timeout -k 10 300 python benchmarks/bench_resnet50_dp.py --steps 10 --warmup 3 > gpurun_out/r50.log 2>&1 || { tail -20 gpurun_out/r50.log; exit 1; }
  grep '^{' gpurun_out/r50.log | cut -c1-160
fi
if [ -n "$ITER_G42" ]; then
  timeout -k 10 200 python bench.py --clients 4 --train-size 25000 --steps 3 --warmup 1 > gpurun_out/hb4.log 2>&1 || { tail -20 gpurun_out/hb4.log; exit 1; }
  grep '^{' gpurun_out/hb4.log | cut -c1-160
  timeout -k 10 200 python bench.py --clients 2 --train-size 12500 --steps 3 --warmup 1 > gpurun_out/hb2.log 2>&1 || { tail -20 gpurun_out/hb2.log; exit 1; }
  grep '^{' gpurun_out/hb2.log | cut -c1-160
fi
