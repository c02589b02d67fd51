#!/bin/bash
# 1-client bench at the standard 6250-sample shard, then the 50000-sample single-client round (crashed in r5y)
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --clients 1 --train-size 6250 --steps 5 --warmup 2 > gpurun_out/r5z_g1.log 2>&1 || { tail -20 gpurun_out/r5z_g1.log; exit 1; }
tail -1 gpurun_out/r5z_g1.log | cut -c1-200
timeout -k 10 300 python -u bench.py --clients 1 --steps 2 --warmup 1 > gpurun_out/r5z_g1big.log 2>&1; rc=$?
echo "big rc=$rc"; tail -30 gpurun_out/r5z_g1big.log | cut -c1-300
