#!/bin/bash
# high-priority capture stream (DDL_GRAPH_PRIO) A/B at 1 and 8 clients on the tuned tables
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
for C in 1 8; do for P in 1 0 1 0; do
  DDL_GRAPH_PRIO=$P timeout -k 10 300 python -u bench.py --clients $C --train-size $((6250 * C)) --steps 5 --warmup 2 > gpurun_out/r5pr_b.log 2>&1 || { tail -5 gpurun_out/r5pr_b.log; exit 1; }
  echo "clients=$C prio=$P $(tail -1 gpurun_out/r5pr_b.log | cut -c95-160)"
done; done
