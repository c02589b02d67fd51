#!/bin/bash
# MnistCnn FedAvg (homework-1 defaults) on the native engine vs the reference loop; lab 1a on GPU.
set -o pipefail
tag=${1:-mn}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -h '^{' "$out/$name.log" | cut -c1-400; tail -n 2 "$out/$name.log" | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
step native 300 python benchmarks/bench_mnist_fedavg.py --variant native --steps 20 --warmup 2
step faithful 300 python benchmarks/bench_mnist_fedavg.py --variant faithful --steps 5 --warmup 1
step lab1a 300 python examples/lab_1a_hfl.py --out $out/lab1a
step prof 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python benchmarks/bench_mnist_fedavg.py --variant native --steps 5 --warmup 2
echo ALLDONE
