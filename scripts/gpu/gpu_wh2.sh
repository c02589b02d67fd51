#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "wgrad" --timeout 120 --timeout-method thread > gpurun_out/tw.log 2>&1 || { tail -30 gpurun_out/tw.log; exit 1; }
tail -1 gpurun_out/tw.log
timeout -k 10 300 python scripts/conv_bench.py --G 8 --layers c64,c128,c256 --wh-splits 8,16,32,64 > gpurun_out/wh8.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/wh8.log | cut -c1-600
timeout -k 10 200 python bench.py --steps 3 --warmup 1 > gpurun_out/hb8.log 2>&1 || exit 1
grep '^{' gpurun_out/hb8.log | cut -c1-160
