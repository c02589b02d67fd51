#!/bin/bash
# deferred presplit on a side stream: halo + fp32 tests, then A/B DDL_F32_PRESPLIT_SIDE at 8 and 1 clients
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_x6h_gpu.py tests/test_fp32_gpu.py > gpurun_out/r5ps_t.log 2>&1; rc=$?
tail -1 gpurun_out/r5ps_t.log; [ $rc = 0 ] || { grep -m5 "Error\|FAILED\|assert" gpurun_out/r5ps_t.log; exit 1; }
for rep in 1 2; do for S in 1 0; do
  DDL_F32_PRESPLIT_SIDE=$S timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/r5ps_g8.log 2>&1 || { tail -5 gpurun_out/r5ps_g8.log; exit 1; }
  echo "side=$S g8 $(tail -1 gpurun_out/r5ps_g8.log | cut -c1-130)"
done; done
for S in 1 0; do
  DDL_F32_PRESPLIT_SIDE=$S timeout -k 10 300 python -u bench.py --clients 1 --train-size 6250 --steps 5 --warmup 2 > gpurun_out/r5ps_g1.log 2>&1 || { tail -5 gpurun_out/r5ps_g1.log; exit 1; }
  echo "side=$S g1 $(tail -1 gpurun_out/r5ps_g1.log | cut -c1-130)"
done
