#!/bin/bash
# side-stream WGRAD overlap (DDL_WGRAD_OVERLAP) A/B at 1 / 2 / 8 clients on the round-5 kernels and plans
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
for C in ${CS:-1 2 8}; do for O in 0 auto 0 auto; do
  DDL_WGRAD_OVERLAP=$O timeout -k 10 300 python -u bench.py --clients $C --train-size $((6250 * C)) --steps 5 --warmup 2 > gpurun_out/r5ov_b.log 2>&1 || { tail -5 gpurun_out/r5ov_b.log; exit 1; }
  echo "clients=$C overlap=$O $(tail -1 gpurun_out/r5ov_b.log | cut -c95-140)"
done; done
