#!/bin/bash
# GPU kernel tests matching a -k filter, then bench.py at 1, 2 and 8 clients (2 reps each).
#   gpurun -- bash scripts/gpu/gpu_quick2.sh <tag> "<pytest -k expr>"
set -o pipefail
tag=${1:-q2}
kexpr=${2:-prep}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -h '^{' "$out/$name.log" | cut -c1-140; tail -n 1 "$out/$name.log" | cut -c1-200
  [ $rc -eq 0 ] || exit $rc
}
step ktests 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$kexpr"
for rep in 1 2; do
  step "c1_$rep" 200 python bench.py --clients 1 --train-size 6250 --steps 4 --warmup 1
  step "c2_$rep" 200 python bench.py --clients 2 --train-size 12500 --steps 3 --warmup 1
  step "c8_$rep" 200 python bench.py --steps 3 --warmup 1
done
echo ALLDONE
