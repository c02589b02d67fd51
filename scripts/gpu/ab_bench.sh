#!/bin/bash
# Headline-bench A/B of kernel-library variants (abvar/<name>.so) at 8 and 1 clients, after the fp32
# GPU tests on the first variant.   bash scripts/gpu/ab_bench.sh "new base" tag
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
VS=${1:-"new base"}; T=${2:-abb}
first=${VS%% *}
DDL_KERNEL_LIB=abvar/$first.so timeout -k 10 600 python -u -m pytest tests/test_fp32_gpu.py -q -x --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for C in 1 8; do for V in $VS; do
  N=$((6250 * C))
  DDL_KERNEL_LIB=abvar/$V.so timeout -k 10 300 python -u bench.py --steps 3 --clients $C --train-size $N > gpurun_out/${T}_${V}_$C.log 2>&1 || { tail -20 gpurun_out/${T}_${V}_$C.log; exit 1; }
  echo "clients=$C $V $(tail -1 gpurun_out/${T}_${V}_$C.log | cut -c1-140)"
done; done
