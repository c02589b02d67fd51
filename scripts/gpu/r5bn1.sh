#!/bin/bash
# one-pass Chan BN finalize: fp32 / halo / FL tests, then 1- and 8-client benches
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_fp32_gpu.py tests/test_kernels_gpu.py tests/test_overlap_gpu.py tests/test_fl_gpu.py > gpurun_out/r5bn1_t.log 2>&1; rc=$?
tail -1 gpurun_out/r5bn1_t.log; [ $rc = 0 ] || { grep -m5 "Error\|FAILED\|assert" gpurun_out/r5bn1_t.log; exit 1; }
for C in 1 8 1 8; do
  timeout -k 10 300 python -u bench.py --clients $C --train-size $((6250 * C)) --steps 5 --warmup 2 > gpurun_out/r5bn1_b.log 2>&1 || { tail -5 gpurun_out/r5bn1_b.log; exit 1; }
  echo "clients=$C $(tail -1 gpurun_out/r5bn1_b.log | cut -c95-140)"
done
