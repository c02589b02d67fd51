#!/bin/bash
# Two round-graph instances (DDL_ROUND_GRAPHS=2) vs one: FL GPU tests, 1/8-client bench A/B, gaps.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/rg2
mkdir -p $out
DDL_ROUND_GRAPHS=2 timeout -k 10 300 python -u -m pytest tests/test_fl_gpu.py tests/test_multirank_gpu.py tests/test_graphs_gpu.py -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
b() { local name=$1; shift; timeout -k 10 300 "$@" > $out/$name.log 2>&1 || { tail -5 $out/$name.log; exit 1; }; echo "$name: $(grep -o '"value": [0-9.]*' $out/$name.log)"; }
for rep in 1 2; do
  for g in 1 2; do
    DDL_ROUND_GRAPHS=$g b c1_g${g}_$rep python bench.py --clients 1 --train-size 6250 --steps 6 --warmup 2
    DDL_ROUND_GRAPHS=$g b c8_g${g}_$rep python bench.py --steps 3 --warmup 1
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/t -o run -- python bench.py --clients 1 --train-size 6250 --steps 4 --warmup 2 > $out/t.log 2>&1 || exit 1
f=$(find $out/t -name '*kernel_trace.csv' | head -1)
python scripts/round_gaps.py "$f" 5
rm -rf $out/t
