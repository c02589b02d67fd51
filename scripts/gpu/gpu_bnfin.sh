#!/bin/bash
# Fused BN finalize+apply A/B: GPU tests, then 1- and 8-client bench alternating
# DDL_BN_FUSED_FIN=0/1, a stripe-count sweep at 1 client, ResNet-50 A/B.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/bnfin
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
b() { local name=$1; shift; timeout -k 10 300 "$@" > $out/$name.log 2>&1 || { tail -5 $out/$name.log; exit 1; }; echo "$name: $(grep -o '"value": [0-9.]*' $out/$name.log)"; }
for rep in 1 2; do
  for f in 0 1; do
    DDL_BN_FUSED_FIN=$f b c1_f${f}_$rep python bench.py --clients 1 --train-size 6250 --steps 5 --warmup 1
    DDL_BN_FUSED_FIN=$f b c8_f${f}_$rep python bench.py --steps 3 --warmup 1
  done
done
for s in 1 2; do DDL_BN_FIN_STRIPES=$s b c1_s$s python bench.py --clients 1 --train-size 6250 --steps 5 --warmup 1; done
for f in 0 1; do DDL_BN_FUSED_FIN=$f b r50_f$f python benchmarks/bench_resnet50_dp.py --steps 10 --warmup 3; done
echo DONE
