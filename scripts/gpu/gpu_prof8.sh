#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/profh
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/h1 -o run -- python bench.py --steps 2 --warmup 1 > $out/h1.log 2>&1 || exit 1
DDL_CONV_HALO=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/h0 -o run -- python bench.py --steps 2 --warmup 1 > $out/h0.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/c1 -o run -- python bench.py --clients 1 --train-size 6250 --steps 3 --warmup 1 > $out/c1.log 2>&1 || exit 1
grep '^{' $out/h1.log $out/h0.log $out/c1.log | cut -c1-150
