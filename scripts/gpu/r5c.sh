#!/bin/bash
# round 5: GAN / tabular device tests, fp32 GAN bench, fp32 LLM bench + kernel profile
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=${1:-r5c}
step() {  # name timeout cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > gpurun_out/${T}_${name}.log 2>&1
  local rc=$?
  echo "[$name] rc=$rc :: $(tail -1 gpurun_out/${T}_${name}.log | cut -c1-400)"
  case $rc in 0) ;; *) echo "[$name] failed: stopping"; tail -40 gpurun_out/${T}_${name}.log; exit 1;; esac
}
for cfg in "A:" "B:DDL_F32_PRESPLIT=0" "C:DDL_F32_PRESPLIT=0 DDL_WGRAD_REDUCE_V4_MIN=0" "D:"; do
  tag=${cfg%%:*}; envs=${cfg#*:}
  step ab$tag 300 env $envs python -u bench.py --steps 5 --warmup 2
done
step gan 300 python -u benchmarks/bench_vfl_gan.py --steps 3 --warmup 2
step llm 300 python -u benchmarks/bench_llm.py --precision fp32 --steps 10 --warmup 3
step llmprof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_llmprof -o run -- python benchmarks/bench_llm.py --precision fp32 --steps 5 --warmup 2
db=$(ls gpurun_out/${T}_llmprof/*/run_results.db gpurun_out/${T}_llmprof/run_results.db 2>/dev/null | head -1)
python scripts/prof_summary.py "$db" --top 30 > gpurun_out/${T}_llmprof_summary.txt
head -34 gpurun_out/${T}_llmprof_summary.txt
rm -rf gpurun_out/${T}_llmprof
step syncdiag 300 python -u scripts/fl_sync_diag.py --reps 2
step mrtests 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_multirank_gpu.py -k "vfl_gan_bench or eight_ranks" -s
