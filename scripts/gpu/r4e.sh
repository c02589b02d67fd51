#!/bin/bash
# BN-backward fold validation + headline bench/profile + MFMA rounding probe + 2-rank fp32 test
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=${1:-r4e}
step() {  # name timeout cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > gpurun_out/${T}_${name}.log 2>&1
  local rc=$?
  echo "[$name] rc=$rc :: $(tail -1 gpurun_out/${T}_${name}.log | cut -c1-300)"
  case $rc in 124|134|137|139) echo "[$name] crashed or timed out: stopping"; exit $rc;; esac
  return 0
}
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
step mfma 60 ./scripts/mfma_rounding.bin
step x6h 300 $PT tests/test_x6h_gpu.py
step fp32 700 $PT tests/test_fp32_gpu.py
step multirank 400 $PT tests/test_multirank_gpu.py -k fp32_resnet18 -s
step bench 300 python -u bench.py --steps 5 --warmup 2
step prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run -- python bench.py --steps 2 --warmup 1
python scripts/prof_summary.py $(ls gpurun_out/${T}_prof/*/run_results.db gpurun_out/${T}_prof/run_results.db 2>/dev/null | head -1) --top 30 > gpurun_out/${T}_prof_summary.txt
head -24 gpurun_out/${T}_prof_summary.txt
cat gpurun_out/${T}_mfma.log
grep -E "fp32 ResNet" gpurun_out/${T}_multirank.log
