#!/bin/bash
# Quick GPU iteration: full GPU test suite, then bench.py at 1, 2 and 8 clients per GPU.
#   gpurun --timeout 900 -- bash scripts/gpu/gpu_quick.sh <tag>
set -o pipefail
tag=${1:-q}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "$out/$name.log" | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
step tests 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step b1 200 python bench.py --clients 1 --train-size 6250 --steps 3 --warmup 1
step b2 200 python bench.py --clients 2 --train-size 12500 --steps 3 --warmup 1
step b8 200 python bench.py --steps 3 --warmup 1
echo ALLDONE
