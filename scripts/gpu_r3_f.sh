#!/bin/bash
# Full GPU suite; headline bench fp32 (tuned plans) / deterministic / bf16; rocprof kernel stats.
set -o pipefail
mkdir -p gpurun_out/prof_f32f
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r3f_gputests.log 2>&1
rc=$?
tail -5 gpurun_out/r3f_gputests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 5 --warmup 1 > gpurun_out/r3f_bench_fp32.log 2>&1 || { tail -20 gpurun_out/r3f_bench_fp32.log; exit 1; }
tail -1 gpurun_out/r3f_bench_fp32.log
timeout -k 10 400 python -u bench.py --steps 5 --warmup 1 --deterministic > gpurun_out/r3f_bench_det.log 2>&1 || { tail -20 gpurun_out/r3f_bench_det.log; exit 1; }
tail -1 gpurun_out/r3f_bench_det.log
timeout -k 10 400 python -u bench.py --steps 5 --warmup 1 --precision bf16 > gpurun_out/r3f_bench_bf16.log 2>&1 || { tail -20 gpurun_out/r3f_bench_bf16.log; exit 1; }
tail -1 gpurun_out/r3f_bench_bf16.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_f32f -o run -- python -u bench.py --steps 3 --warmup 1 \
  > gpurun_out/r3f_prof.log 2>&1 || { tail -20 gpurun_out/r3f_prof.log; exit 1; }
tail -1 gpurun_out/r3f_prof.log
db=$(ls gpurun_out/prof_f32f/*/run_results.db gpurun_out/prof_f32f/run_results.db 2>/dev/null | head -n 1 || true)
[ -n "$db" ] && python scripts/prof_summary.py "$db" --top 40 > gpurun_out/r3f_prof_summary.txt
exit 0
