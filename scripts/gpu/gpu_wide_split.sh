#!/bin/bash
# wide split-K FWD/DGRAD tuner candidates: explicit-tile tests first (bounded), then 1/2-client bench A/B
# (DDL_TUNE_WIDE_SPLIT=0/1 alternating) and a 1-client step trace with them.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/widesplit
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "split" > $out/t1.log 2>&1 || { tail -30 $out/t1.log; exit 1; }
tail -1 $out/t1.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
b() { local name=$1; shift; timeout -k 10 300 "$@" > $out/$name.log 2>&1 || { tail -5 $out/$name.log; exit 1; }; echo "$name: $(grep -o '"value": [0-9.]*' $out/$name.log)"; }
for rep in 1 2; do
  for h in 0 1; do
    DDL_TUNE_WIDE_SPLIT=$h b c1_h${h}_$rep python bench.py --clients 1 --train-size 6250 --steps 5 --warmup 1
    DDL_TUNE_WIDE_SPLIT=$h b c2_h${h}_$rep python bench.py --clients 2 --train-size 12500 --steps 4 --warmup 1
  done
done
DDL_TUNE_WIDE_SPLIT=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/c1 -o run -- python bench.py --clients 1 --train-size 6250 --steps 2 --warmup 1 > $out/c1.log 2>&1 || exit 1
f=$(find $out/c1 -name '*kernel_trace.csv' | head -1)
python scripts/step_trace.py $f > $out/step_c1.txt && rm -rf $out/c1
grep "conv_" $out/step_c1.txt | head -20
tail -1 $out/step_c1.txt
