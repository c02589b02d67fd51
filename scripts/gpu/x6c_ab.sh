#!/bin/bash
# conv_x6h chain length A/B in one box: default library (2-step chains) vs build/ab (1-step)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
DDL_KERNEL_LIB=$PWD/ddl25spring_amd/lib/ab/libddl_kernels_ch3.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_x6h_gpu.py tests/test_fp32_gpu.py > gpurun_out/x6c3_tests.log 2>&1; rc=$?; echo "ch3 tests rc=$rc: $(tail -1 gpurun_out/x6c3_tests.log)"
case $rc in 0|1) ;; *) exit 1;; esac
for M in fwd dgrad; do for L in c64 c128 c256; do for V in 2 3; do
  if [ $V != 2 ]; then export DDL_KERNEL_LIB=$PWD/ddl25spring_amd/lib/ab/libddl_kernels_ch$V.so; else unset DDL_KERNEL_LIB; fi
  timeout -k 10 60 python scripts/conv_f32_bench.py --math auto --mode $M --layer $L --reps 20 2>&1 | tail -1 | sed "s/^/chain=$V /" || exit 1
done; done; done
for V in 2 3 2 3; do
  if [ $V != 2 ]; then export DDL_KERNEL_LIB=$PWD/ddl25spring_amd/lib/ab/libddl_kernels_ch$V.so; else unset DDL_KERNEL_LIB; fi
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_ch$V.json 2> gpurun_out/bench_ch$V.err || exit 1
  echo "chain=$V $(tail -1 gpurun_out/bench_ch$V.json | cut -c100-160)"
done
