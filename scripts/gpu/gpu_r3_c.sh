#!/bin/bash
# fp32 path: full GPU test suite, headline bench with tuned plans, rocprof kernel stats, tuning G=4/2.
set -o pipefail
mkdir -p gpurun_out/prof_f32
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r3_gputests.log 2>&1
rc=$?
tail -5 gpurun_out/r3_gputests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 > gpurun_out/r3_bench_fp32_tuned.log 2>&1 || { tail -20 gpurun_out/r3_bench_fp32_tuned.log; exit 1; }
tail -1 gpurun_out/r3_bench_fp32_tuned.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_f32 -o run -- python -u bench.py --steps 2 --warmup 1 \
  > gpurun_out/r3_prof_f32.log 2>&1 || { tail -20 gpurun_out/r3_prof_f32.log; exit 1; }
tail -1 gpurun_out/r3_prof_f32.log
timeout -k 10 420 python -u scripts/conv_f32_tune.py --out gpurun_out/f32_plans_g42.json --groups 4 2 --budget-s 360 \
  > gpurun_out/r3_tune_g42.log 2>&1
tail -2 gpurun_out/r3_tune_g42.log
