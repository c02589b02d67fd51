#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tk.log 2>&1; rc=$?; tail -3 gpurun_out/tk.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/conv_bench.py --G 8 --epi > gpurun_out/ee8.log 2>&1 && grep -v amdgpu.ids gpurun_out/ee8.log &&
timeout -k 10 300 python scripts/conv_bench.py --G 1 --epi > gpurun_out/ee1.log 2>&1 && grep -v amdgpu.ids gpurun_out/ee1.log &&
timeout -k 10 200 python bench.py --steps 3 --warmup 1 > gpurun_out/hb8.log 2>&1 && grep '^{' gpurun_out/hb8.log | cut -c1-200 &&
timeout -k 10 200 python bench.py --clients 1 --train-size 6250 --steps 3 --warmup 1 > gpurun_out/hb1.log 2>&1 && grep '^{' gpurun_out/hb1.log | cut -c1-200
