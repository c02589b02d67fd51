#!/bin/bash
# 1-client kernel trace: per-kernel totals + per-step gaps/busy (after the slice-outer split-K fold)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r5tr}
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${T}_trace1 -o run -- python bench.py --steps 1 --warmup 1 --clients 1 --train-size 6250 > gpurun_out/${T}_trace.log 2>&1 || { tail -20 gpurun_out/${T}_trace.log; exit 1; }
db=$(ls gpurun_out/${T}_trace1/*/run_results.db gpurun_out/${T}_trace1/run_results.db 2>/dev/null | head -1)
python scripts/step_trace_db.py "$db" > gpurun_out/${T}_step1.txt
python scripts/prof_summary.py "$db" --top 45 > gpurun_out/${T}_top1.txt
tail -3 gpurun_out/${T}_step1.txt
rm -rf gpurun_out/${T}_trace1
