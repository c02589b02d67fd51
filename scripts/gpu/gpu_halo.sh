#!/bin/bash
# Halo conv iteration: halo numerics first, then all kernel tests, per-layer sweep incl. halo tiles, bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -v -k halo --timeout 120 --timeout-method thread > gpurun_out/th.log 2>&1; rc=$?; tail -8 gpurun_out/th.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tk.log 2>&1 && tail -1 gpurun_out/tk.log &&
timeout -k 10 300 python scripts/conv_bench.py --G 8 --sweep --layers c64,c128,c256,c512 > gpurun_out/hs8.log 2>&1 &&
timeout -k 10 300 python scripts/conv_bench.py --G 1 --sweep --layers c64,c128,c256,c512 > gpurun_out/hs1.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 3 --warmup 1 > gpurun_out/hb8.log 2>&1 && grep '^{' gpurun_out/hb8.log | cut -c1-200 &&
timeout -k 10 200 python bench.py --clients 1 --train-size 6250 --steps 3 --warmup 1 > gpurun_out/hb1.log 2>&1 && grep '^{' gpurun_out/hb1.log | cut -c1-200 &&
DDL_CONV_HALO=0 timeout -k 10 200 python bench.py --steps 3 --warmup 1 > gpurun_out/hb8_nohalo.log 2>&1 && grep '^{' gpurun_out/hb8_nohalo.log | cut -c1-200
