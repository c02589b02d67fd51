#!/bin/bash
# bench.py at 1, 2, 4 and 8 clients on one GPU: the per-GPU load of the N = 8, 4, 2, 1 strong-
# scaling runs (8 clients in total over N GPUs).
set -o pipefail
out=gpurun_out/${1:-sweep}
mkdir -p $out
for c in 1 2 4 8; do
  n=$((6250 * c))
  timeout -k 10 300 python bench.py --clients $c --train-size $n --steps 3 --warmup 1 > $out/c$c.log 2>&1 || { tail -5 $out/c$c.log; exit 1; }
  echo "c$c $(grep -h '^{' $out/c$c.log | cut -c1-140)"
done
