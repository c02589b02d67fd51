#!/bin/bash
# Quick GPU iteration: kernel/engine tests, then the headline bench at 8 clients and 1 client.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_overlap_gpu.py tests/test_fl_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/t2.log 2>&1 && tail -3 gpurun_out/t2.log &&
timeout -k 10 200 python bench.py --steps 3 --warmup 1 2>&1 | grep '^{' | cut -c1-200 &&
timeout -k 10 200 python bench.py --clients 1 --train-size 6250 --steps 3 --warmup 1 2>&1 | grep '^{' | cut -c1-200
