#!/bin/bash
# Whole-round HIP graph + fused label gather: GPU FL/kernel tests, then bench at 1, 2, 8 clients;
# fused BN tails with a small re-read budget (DDL_BN_FUSED_BYTES) at 1 and 2 clients.
set -o pipefail
tag=${1:-rg}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -h '^{' "$out/$name.log" | cut -c1-150; tail -n 1 "$out/$name.log" | cut -c1-200
  [ $rc -eq 0 ] || exit $rc
}
step tests 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
for rep in 1 2; do
  step "c1_$rep" 200 python bench.py --clients 1 --train-size 6250 --steps 4 --warmup 1
  step "c2_$rep" 200 python bench.py --clients 2 --train-size 12500 --steps 3 --warmup 1
  step "c8_$rep" 200 python bench.py --steps 3 --warmup 1
  step "c1f4_$rep" 200 env DDL_BN_FUSED_TAIL=auto DDL_BN_FUSED_BYTES=4194304 python bench.py --clients 1 --train-size 6250 --steps 4 --warmup 1
  step "c1f1_$rep" 200 env DDL_BN_FUSED_TAIL=auto DDL_BN_FUSED_BYTES=1048576 python bench.py --clients 1 --train-size 6250 --steps 4 --warmup 1
done
echo ALLDONE
