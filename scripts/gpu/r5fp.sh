#!/bin/bash
# final round-5 kernel profiles: 8-client and 1-client kernel stats + 8-client step trace
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=r5fp
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/${T}_t8 -o run -- python bench.py --steps 1 --warmup 1 > gpurun_out/${T}_t8.log 2>&1 || { tail -20 gpurun_out/${T}_t8.log; exit 1; }
db=$(ls gpurun_out/${T}_t8/*/run_results.db gpurun_out/${T}_t8/run_results.db 2>/dev/null | head -1)
python scripts/step_trace_db.py "$db" > gpurun_out/${T}_step8.txt
python scripts/prof_summary.py "$db" --top 45 > gpurun_out/${T}_top8.txt
tail -1 gpurun_out/${T}_step8.txt; head -12 gpurun_out/${T}_top8.txt
rm -rf gpurun_out/${T}_t8
