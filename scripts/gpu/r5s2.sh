#!/bin/bash
# slice-outer split-K epilogue fold: fp32 + halo tests, then 1 / 8 client benches
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_fp32_gpu.py tests/test_x6h_gpu.py > gpurun_out/r5s2_t.log 2>&1; rc=$?
tail -1 gpurun_out/r5s2_t.log; [ $rc = 0 ] || { grep -m5 "Error\|FAILED\|assert" gpurun_out/r5s2_t.log; exit 1; }
timeout -k 10 300 python -u bench.py --clients 1 --train-size 6250 --steps 5 --warmup 2 > gpurun_out/r5s2_g1.log 2>&1 || { tail -5 gpurun_out/r5s2_g1.log; exit 1; }
echo "g1 $(tail -1 gpurun_out/r5s2_g1.log | cut -c1-200)"
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/r5s2_g8.log 2>&1 || { tail -5 gpurun_out/r5s2_g8.log; exit 1; }
echo "g8 $(tail -1 gpurun_out/r5s2_g8.log | cut -c1-200)"
