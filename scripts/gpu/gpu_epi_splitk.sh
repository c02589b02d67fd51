#!/bin/bash
# Split-K epilogue change: numerics tests, then the 1-client headline under rocprofv3 --stats.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/esk
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "split or conv_dgrad or conv_fwd" > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof1 -o run -- python bench.py --clients 1 --train-size 6250 --steps 3 --warmup 1 > $out/prof1.log 2>&1 || { tail -20 $out/prof1.log; exit 1; }
grep '^{' $out/prof1.log | cut -c1-200
timeout -k 10 300 python bench.py --clients 1 --train-size 6250 --steps 5 --warmup 1 > $out/h1.log 2>&1 || { tail -20 $out/h1.log; exit 1; }
grep '^{' $out/h1.log | cut -c1-200
echo DONE
