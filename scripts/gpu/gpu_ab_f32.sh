#!/bin/bash
# A/B of fp32 conv kernel library variants (abvar/<name>.so): per-layer micro-bench for the listed
# modes, fp32 numerics tests and the headline bench on the first variant.
#   bash scripts/gpu/gpu_ab_f32.sh "tapin tapout" "fwd dgrad" "c64 c128 c256 c512 c128s2" tag
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
VS=${1:-"tapin tapout"}; MO=${2:-"fwd dgrad wgrad"}; LS=${3:-"c64 c256 c128s2"}; T=${4:-ab}
first=${VS%% *}
DDL_KERNEL_LIB=abvar/$first.so timeout -k 10 600 python -u -m pytest tests/test_fp32_gpu.py -q -x --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for V in $VS; do
  for L in $LS; do for O in $MO; do
    echo -n "$V " >> gpurun_out/${T}_layers.log
    DDL_KERNEL_LIB=abvar/$V.so timeout -k 10 60 python scripts/conv_f32_bench.py --math x6 --mode $O --layer $L --reps 20 2>/dev/null >> gpurun_out/${T}_layers.log || { tail -5 gpurun_out/${T}_layers.log; exit 1; }
  done; done
done
cat gpurun_out/${T}_layers.log
for V in $VS; do
  DDL_KERNEL_LIB=abvar/$V.so timeout -k 10 300 python -u bench.py --steps 3 > gpurun_out/${T}_bench_$V.log 2>&1 || { tail -20 gpurun_out/${T}_bench_$V.log; exit 1; }
  echo "$V $(tail -1 gpurun_out/${T}_bench_$V.log | cut -c1-150)"
done
