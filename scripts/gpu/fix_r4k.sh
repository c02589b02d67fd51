#!/bin/bash
# re-run the two failures of the full GPU run, then accuracy with the halo WGRAD off (chain-3 only)
set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k robust_kernels tests/test_multirank_gpu.py -k "robust_kernels or fp32_resnet18" -s > gpurun_out/fix_r4k.log 2>&1; rc=$?
grep -E "passed|failed|rel\(w\)|Error" gpurun_out/fix_r4k.log | tail -5
case $rc in 0|1) ;; *) exit 1;; esac
for cfg in "1 50" "1 100"; do
  set -- $cfg
  DDL_F32_HALO_WGRAD=0 timeout -k 10 120 python scripts/debug_r18_grads.py --quiet --groups $1 --batch $2 2>&1 | grep -v amdgpu.ids | tail -3 | cut -c1-200 || exit 1
done
