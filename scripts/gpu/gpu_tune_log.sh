#!/bin/bash
# Tuner candidate timings of the 8-client headline step, direct SGD off / on (stderr [tune] lines).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/tunelog
mkdir -p $out
for d in 0 1 0 1; do
  DDL_TUNE_LOG=1 DDL_DIRECT_SGD=$d timeout -k 10 300 python bench.py --steps 2 --warmup 1 > $out/b8_d$d.log 2>&1 || { tail -5 $out/b8_d$d.log; exit 1; }
  echo "direct=$d $(grep -o '"value": [0-9.]*' $out/b8_d$d.log)"
  grep "\[tune\] ('wgrad', 8, 100, 32, 32, 64, 64" $out/b8_d$d.log | head -40
done
