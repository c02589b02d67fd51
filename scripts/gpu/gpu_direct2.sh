#!/bin/bash
# Direct SGD with the declaration-order layout + direct map: GPU tests, then headline (8 / 1
# clients) and MnistCnn FedAvg A/B with DDL_DIRECT_SGD=0/1 alternating.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/direct2
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
b() { local name=$1; shift; timeout -k 10 300 "$@" > $out/$name.log 2>&1 || { tail -5 $out/$name.log; exit 1; }; echo "$name: $(grep -o '"value": [0-9.]*' $out/$name.log)"; }
for rep in 1 2; do
  for d in 0 1; do
    DDL_DIRECT_SGD=$d b c8_d${d}_$rep python bench.py --steps 3 --warmup 1
    DDL_DIRECT_SGD=$d b c1_d${d}_$rep python bench.py --clients 1 --train-size 6250 --steps 5 --warmup 1
    DDL_DIRECT_SGD=$d b mnist_d${d}_$rep python benchmarks/bench_mnist_fedavg.py --steps 20 --warmup 2
  done
done
echo DONE
