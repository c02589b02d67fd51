#!/bin/bash
# fp32 LLaMA kernel totals (rocprofv3 kernel trace of the LLM bench)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r5llmp}
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${T}_t -o run -- python ${PROF_CMD:-benchmarks/bench_llm.py --precision fp32 --steps 5 --warmup 2} > gpurun_out/${T}.log 2>&1 || { tail -20 gpurun_out/${T}.log; exit 1; }
db=$(ls gpurun_out/${T}_t/*/run_results.db gpurun_out/${T}_t/run_results.db 2>/dev/null | head -1)
python scripts/prof_summary.py "$db" --top 40 > gpurun_out/${T}_top.txt
head -30 gpurun_out/${T}_top.txt | cut -c1-150
rm -rf gpurun_out/${T}_t
