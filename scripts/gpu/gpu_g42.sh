#!/bin/bash
# per-GPU loads of the N=2 and N=4 scaling runs (4 and 2 clients per GPU): halo sweeps + bench
set -o pipefail
mkdir -p gpurun_out
for G in 4 2; do
  timeout -k 10 300 python scripts/conv_bench.py --G $G --sweep --epi --layers c64,c128 --wh-splits 8,16,32,64,128 > gpurun_out/g$G.log 2>&1 || { tail -20 gpurun_out/g$G.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/g$G.log | cut -c1-900
done
timeout -k 10 200 python bench.py --clients 4 --train-size 25000 --steps 3 --warmup 1 > gpurun_out/hb4.log 2>&1 || exit 1
grep '^{' gpurun_out/hb4.log | cut -c1-200
timeout -k 10 200 python bench.py --clients 2 --train-size 12500 --steps 3 --warmup 1 > gpurun_out/hb2.log 2>&1 || exit 1
grep '^{' gpurun_out/hb2.log | cut -c1-200
