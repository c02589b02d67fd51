#!/bin/bash
# Conv iteration: conv kernel tests, per-layer conv timings at 8 and 1 clients, headline bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tk.log 2>&1 && tail -1 gpurun_out/tk.log &&
timeout -k 10 200 python scripts/conv_bench.py --G 8 > gpurun_out/cb8.log 2>&1 && grep -v amdgpu.ids gpurun_out/cb8.log &&
timeout -k 10 200 python scripts/conv_bench.py --G 1 > gpurun_out/cb1.log 2>&1 && grep -v amdgpu.ids gpurun_out/cb1.log &&
timeout -k 10 200 python bench.py --steps 3 --warmup 1 2>&1 | grep '^{' | cut -c1-160 &&
timeout -k 10 200 python bench.py --clients 1 --train-size 6250 --steps 3 --warmup 1 2>&1 | grep '^{' | cut -c1-160
