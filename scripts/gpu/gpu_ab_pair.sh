#!/bin/bash
# A/B of the paired DGRAD+WGRAD launches: conv GPU tests, then bench.py at 1 and 8 clients per GPU
# with pairing on (default) and off (DDL_CONV_PAIR=0).
#   gpurun --timeout 900 -- bash scripts/gpu/gpu_ab_pair.sh
set -o pipefail
out=gpurun_out/pair
mkdir -p $out
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "$out/$name.log" | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
}
step tests 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "conv"
step b1_on 200 python bench.py --clients 1 --train-size 6250 --steps 3 --warmup 1
step b1_off 200 env DDL_CONV_PAIR=0 python bench.py --clients 1 --train-size 6250 --steps 3 --warmup 1
step b8_on 200 python bench.py --steps 3 --warmup 1
step b8_off 200 env DDL_CONV_PAIR=0 python bench.py --steps 3 --warmup 1
step b2_on 200 python bench.py --clients 2 --train-size 12500 --steps 3 --warmup 1
step b2_off 200 env DDL_CONV_PAIR=0 python bench.py --clients 2 --train-size 12500 --steps 3 --warmup 1
echo ALLDONE
