#!/bin/bash
# Headline-bench A/B of an environment switch at 8 and 1 clients:  bash scripts/gpu/ab_env.sh VAR "v1 v0" tag
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
VAR=$1; VS=${2:-"1 0"}; T=${3:-abenv}
for C in 1 8; do for V in $VS; do
  N=$((6250 * C))
  env $VAR=$V timeout -k 10 300 python -u bench.py --steps 3 --clients $C --train-size $N > gpurun_out/${T}_${V}_$C.log 2>&1 || { tail -20 gpurun_out/${T}_${V}_$C.log; exit 1; }
  echo "clients=$C $VAR=$V $(tail -1 gpurun_out/${T}_${V}_$C.log | cut -c1-140)"
done; done
