#!/bin/bash
# LLaMA fp32: one step's kernels in order (kernel trace)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=${1:-r5r}
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/${T}_llm -o run -- python benchmarks/bench_llm.py --precision fp32 --steps 4 --warmup 2 > gpurun_out/${T}_llm.log 2>&1 || { tail -20 gpurun_out/${T}_llm.log; exit 1; }
db=$(ls gpurun_out/${T}_llm/*/run_results.db gpurun_out/${T}_llm/run_results.db 2>/dev/null | head -1)
STEP_MARK=adam_ python scripts/step_trace_db.py "$db" > gpurun_out/${T}_llm_step.txt
python scripts/prof_summary.py "$db" --top 30 > gpurun_out/${T}_llm_top.txt
tail -1 gpurun_out/${T}_llm_step.txt
rm -rf gpurun_out/${T}_llm
