#!/bin/bash
# One client per GPU (the per-GPU load of the 8-GPU headline run): kernel-stats profile + per-layer G=1 timings.
set -o pipefail
mkdir -p gpurun_out/prof_g1
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_g1 -o run -- python -u bench.py --clients 1 --train-size 6250 --steps 3 --warmup 1 \
  > gpurun_out/prof_g1.log 2>&1 || { tail -20 gpurun_out/prof_g1.log; exit 1; }
tail -1 gpurun_out/prof_g1.log | cut -c1-200
db=$(ls gpurun_out/prof_g1/*/run_results.db gpurun_out/prof_g1/run_results.db 2>/dev/null | head -n 1 || true)
[ -n "$db" ] && python scripts/prof_summary.py "$db" --top 40 > gpurun_out/prof_g1_summary.txt
head -42 gpurun_out/prof_g1_summary.txt
for L in c64 c128 c256 c512 c128s2 sc128; do for O in fwd dgrad wgrad; do
  timeout -k 10 60 python scripts/conv_f32_bench.py --math x6 --mode $O --layer $L --G 1 --reps 50 2>/dev/null >> gpurun_out/g1_layers.log || exit 1
done; done
cat gpurun_out/g1_layers.log
