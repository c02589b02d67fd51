#!/bin/bash
# round 6 evidence: fp32 gradient accuracy of this tree (batch 16 / 50 / 100) and the 8-rank
# rehearsals (pinned plans: bitwise the single process; tuned plans: rank hashes equal)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=${1:-r6e}
for b in 16 50 100; do
  echo "== batch $b" >> gpurun_out/${T}_acc.txt
  timeout -k 10 200 python -u scripts/debug_r18_grads.py --batch $b --quiet >> gpurun_out/${T}_acc.txt 2>&1 || { tail -5 gpurun_out/${T}_acc.txt; exit 1; }
done
cat gpurun_out/${T}_acc.txt | cut -c1-200
timeout -k 10 900 python -u -m pytest tests/test_multirank_gpu.py -x -v -s -k "eight_ranks" --timeout 850 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_8rank.log 2>&1
rc=$?; grep -E "PASSED|FAILED|passed|failed|^\{" gpurun_out/${T}_8rank.log | cut -c1-400; exit $rc
