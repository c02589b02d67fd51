#!/bin/bash
# A/B of one env switch (0 vs 1) on bench.py at 1 and 8 clients, after the GPU tests matching -k.
#   gpurun -- bash scripts/gpu/gpu_ab.sh <tag> <ENV_VAR> "<pytest -k expr>"
set -o pipefail
tag=${1:-ab}
var=${2:-DDL_FUSED_HEAD}
kexpr=${3:-head}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc $(grep -h '^{' "$out/$name.log" | cut -c1-110) $(tail -n 1 "$out/$name.log" | cut -c1-80)"
  [ $rc -eq 0 ] || { tail -n 30 "$out/$name.log"; exit $rc; }
}
step ktests 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$kexpr"
for rep in 1 2; do
  for v in 0 1; do
    step "c1_${v}_$rep" 200 env $var=$v python bench.py --clients 1 --train-size 6250 --steps 4 --warmup 1
    step "c8_${v}_$rep" 200 env $var=$v python bench.py --steps 3 --warmup 1
  done
done
echo ALLDONE
