#!/bin/bash
# Fused BN tails: GPU tests, then bench.py A/B (DDL_BN_FUSED_TAIL=0 vs auto) at 1, 2, 8 clients.
#   gpurun --timeout 900 -- bash scripts/gpu/gpu_ab_bntail.sh <tag>
set -o pipefail
tag=${1:-bt}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -h '^{' "$out/$name.log" | cut -c1-200; tail -n 2 "$out/$name.log" | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
step tests 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "fused_tails or bn"
for rep in 1 2; do
  for mode in 0 auto; do
    step "c1_${mode}_$rep" 200 env DDL_BN_FUSED_TAIL=$mode python bench.py --clients 1 --train-size 6250 --steps 4 --warmup 1
    step "c2_${mode}_$rep" 200 env DDL_BN_FUSED_TAIL=$mode python bench.py --clients 2 --train-size 12500 --steps 3 --warmup 1
    step "c8_${mode}_$rep" 200 env DDL_BN_FUSED_TAIL=$mode python bench.py --steps 3 --warmup 1
  done
done
echo ALLDONE
