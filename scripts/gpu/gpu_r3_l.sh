#!/bin/bash
# A/B of X6 accumulation variants (abvar/*.so): per-layer micro-bench, fp32 numerics on the
# chained variant, headline bench per variant.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for V in base ch1 ch2; do
  for L in c64 c128 c256 c512 c128s2; do for O in fwd dgrad wgrad; do
    echo -n "$V " >> gpurun_out/r3l_layers.log
    DDL_KERNEL_LIB=abvar/$V.so timeout -k 10 60 python scripts/conv_f32_bench.py --math x6 --mode $O --layer $L --reps 20 2>/dev/null >> gpurun_out/r3l_layers.log || { tail -5 gpurun_out/r3l_layers.log; exit 1; }
  done; done
done
cat gpurun_out/r3l_layers.log
DDL_KERNEL_LIB=abvar/ch2.so timeout -k 10 600 python -u -m pytest tests/test_fp32_gpu.py -q -x --timeout 300 --timeout-method thread > gpurun_out/r3l_tests.log 2>&1 || { tail -30 gpurun_out/r3l_tests.log; exit 1; }
tail -2 gpurun_out/r3l_tests.log
for V in base ch1 ch2; do
  DDL_KERNEL_LIB=abvar/$V.so timeout -k 10 300 python -u bench.py --steps 3 > gpurun_out/r3l_bench_$V.log 2>&1 || { tail -20 gpurun_out/r3l_bench_$V.log; exit 1; }
  echo "$V $(tail -1 gpurun_out/r3l_bench_$V.log | cut -c1-160)"
done
