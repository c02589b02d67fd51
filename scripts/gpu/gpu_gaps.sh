#!/bin/bash
# Per-round GPU idle time of the 1- and 8-client bench (kernel trace of 4 timed rounds).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/gaps
mkdir -p $out
for c in 1 8; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/t$c -o run -- python bench.py --clients $c --train-size $((6250 * c)) --steps 4 --warmup 2 > $out/t$c.log 2>&1 || exit 1
  f=$(find $out/t$c -name '*kernel_trace.csv' | head -1)
  echo "== $c client(s)"
  python scripts/round_gaps.py "$f" 5 | tee $out/gaps$c.txt
  rm -rf $out/t$c
done
