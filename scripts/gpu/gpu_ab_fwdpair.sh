#!/bin/bash
# FWD+FWD conv pairing A/B (DDL_CONV_PAIR_FWD=0 vs 1) after the pair kernel tests.
set -o pipefail
tag=${1:-fwdpair}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc $(grep -h '^{' "$out/$name.log" | cut -c1-110)"
  [ $rc -eq 0 ] || { tail -n 5 "$out/$name.log"; exit $rc; }
}
step ktests 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "pair or resnet or fusion"
for rep in 1 2; do
  for v in 0 1; do
    step "c1_p${v}_$rep" 200 env DDL_CONV_PAIR_FWD=$v python bench.py --clients 1 --train-size 6250 --steps 4 --warmup 1
    step "c8_p${v}_$rep" 200 env DDL_CONV_PAIR_FWD=$v python bench.py --steps 3 --warmup 1
  done
done
echo ALLDONE
