#!/bin/bash
# One gpurun call: GPU tests, headline bench (8 clients and the per-GPU load of the N=8 run),
# reference-equivalent eager baselines, and a rocprofv3 kernel-stats profile of bench.py.
#   gpurun --timeout 1200 -- bash scripts/gpu/gpu_check.sh [tests|bench|prof|all]
set -o pipefail
what=${1:-all}
out=gpurun_out
mkdir -p $out
export TMPDIR=/tmp
step() {  # step <name> <seconds> <cmd...>: stop the whole script on the first failure
  local name=$1 secs=$2; shift 2
  echo "== $name" | tee -a $out/steps.txt
  timeout -k 10 "$secs" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $out/steps.txt
  tail -3 "$out/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
if [ "$what" = tests ] || [ "$what" = all ]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
fi
if [ "$what" = bench ] || [ "$what" = all ]; then
  step bench8 300 python bench.py --steps 3 --warmup 1
  step bench1client 300 python bench.py --clients 1 --train-size 6250 --steps 3 --warmup 1
  step eager_tuned 400 python benchmarks/bench_reference_eager.py --variant tuned --steps 1 --warmup 1
  step eager_faithful 600 python benchmarks/bench_reference_eager.py --variant faithful --steps 1 --warmup 0
fi
if [ "$what" = prof ] || [ "$what" = all ]; then
  step prof8 300 rocprofv3 --kernel-trace --stats -d $out/prof8 -o run -- python bench.py --steps 2 --warmup 1
  step prof1 300 rocprofv3 --kernel-trace --stats -d $out/prof1 -o run -- python bench.py --clients 1 --train-size 6250 --steps 2 --warmup 1
fi
echo ALLDONE
