#!/bin/bash
# Direct SGD A/B: GPU FL tests, then the headline bench at 8 and 1 clients with DDL_DIRECT_SGD=0/1
# alternating, then a kernel-stats profile of the direct path (summaries only, raw traces removed).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/direct
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_fl_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for rep in 1 2; do
  for d in 0 1; do
    DDL_DIRECT_SGD=$d timeout -k 10 300 python bench.py --steps 3 --warmup 1 > $out/b8_d${d}_$rep.log 2>&1 || { tail -5 $out/b8_d${d}_$rep.log; exit 1; }
    echo "8 clients direct=$d: $(grep -o '"value": [0-9.]*' $out/b8_d${d}_$rep.log)"
    DDL_DIRECT_SGD=$d timeout -k 10 300 python bench.py --clients 1 --train-size 6250 --steps 5 --warmup 1 > $out/b1_d${d}_$rep.log 2>&1 || { tail -5 $out/b1_d${d}_$rep.log; exit 1; }
    echo "1 client  direct=$d: $(grep -o '"value": [0-9.]*' $out/b1_d${d}_$rep.log)"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof8 -o run -- python bench.py --steps 2 --warmup 1 > $out/prof8.log 2>&1 || { tail -5 $out/prof8.log; exit 1; }
f=$(find $out/prof8 -name '*kernel_stats.csv' | head -1)
python scripts/prof_summary.py "$f" 30 > $out/prof8_summary.txt && cp "$f" $out/prof8_kernel_stats.csv
rm -rf $out/prof8
head -12 $out/prof8_summary.txt
echo DONE
