#!/bin/bash
# round 6: the single-client 50,000-sample ResNet-18 round (500 local steps) with the round graph
# chunked at $1 steps (DDL_GRAPH_MAX_STEPS); round 5 saw the 500-step whole-round graph segfault in
# hipGraphLaunch. One value per call: a crash ends the call (no retry on the GPU).
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
N=${1:-256}
T=${2:-r6gb}
DDL_GRAPH_MAX_STEPS=$N timeout -k 10 400 python -u bench.py --clients 1 --steps 2 --warmup 1 > gpurun_out/${T}_${N}.log 2>&1
rc=$?
echo "chunk=$N rc=$rc"
grep -E '^\{' gpurun_out/${T}_${N}.log | cut -c1-200
[ $rc -eq 0 ] || tail -15 gpurun_out/${T}_${N}.log | cut -c1-200
exit $rc
