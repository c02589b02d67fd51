#!/bin/bash
# Big-halo WGRAD tuning rule A/B at 8 and 4 clients (alternating), then a per-launch trace at 8.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/tuneab
mkdir -p $out
for rep in 1 2; do
  for t in 1 0; do
    DDL_TUNE_BIG_HALO=$t timeout -k 10 300 python bench.py --steps 3 --warmup 1 > $out/b8_$t.log 2>&1 || { tail -5 $out/b8_$t.log; exit 1; }
    echo "8 clients tune_big_halo=$t: $(grep -o '"value": [0-9.]*' $out/b8_$t.log)"
    DDL_TUNE_BIG_HALO=$t timeout -k 10 300 python bench.py --clients 4 --train-size 25000 --steps 3 --warmup 1 > $out/b4_$t.log 2>&1 || { tail -5 $out/b4_$t.log; exit 1; }
    echo "4 clients tune_big_halo=$t: $(grep -o '"value": [0-9.]*' $out/b4_$t.log)"
  done
done
bash scripts/gpu/gpu_trace1.sh r2j > /dev/null 2>&1 || exit 1
tail -n 1 gpurun_out/r2j/step_c1.txt gpurun_out/r2j/step_c8.txt
