#!/bin/bash
# A/B of two kernel-library builds (new in-tree vs scratch/ab/libddl_kernels_prev.so): kernel
# tests on the new one, then the headline bench alternating builds.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tk.log 2>&1 || { tail -30 gpurun_out/tk.log; exit 1; }
tail -1 gpurun_out/tk.log
for i in 1 2; do
  for v in new prev; do
    if [ $v = prev ]; then export DDL_KERNEL_LIB=$PWD/scratch/ab/libddl_kernels_prev.so; else unset DDL_KERNEL_LIB; fi
    timeout -k 10 200 python bench.py --steps 3 --warmup 1 ${AB_ARGS} > gpurun_out/ab_$v$i.log 2>&1 || { tail -20 gpurun_out/ab_$v$i.log; exit 1; }
    echo "$v$i $(grep -o '"value": [0-9.]*' gpurun_out/ab_$v$i.log)"
  done
done
