#!/bin/bash
# Round-end numbers: clients-per-GPU sweep (8/4/2/1 = the per-GPU load of N = 1/2/4/8 GPUs) and the
# headline kernel profile.
set -o pipefail
mkdir -p gpurun_out/prof_final
export PYTHONUNBUFFERED=1
for C in 8 4 2 1; do
  T=$((6250 * C))
  timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --clients $C --train-size $T >> gpurun_out/final_sweep.jsonl 2> gpurun_out/final_sweep_$C.err || { tail -20 gpurun_out/final_sweep_$C.err; exit 1; }
  tail -1 gpurun_out/final_sweep.jsonl | cut -c1-160
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_final -o run -- python -u bench.py --steps 3 --warmup 1 \
  > gpurun_out/final_prof.log 2>&1 || { tail -20 gpurun_out/final_prof.log; exit 1; }
db=$(ls gpurun_out/prof_final/*/run_results.db gpurun_out/prof_final/run_results.db 2>/dev/null | head -n 1 || true)
[ -n "$db" ] && python scripts/prof_summary.py "$db" --top 30 > gpurun_out/final_prof_summary.txt
head -12 gpurun_out/final_prof_summary.txt
