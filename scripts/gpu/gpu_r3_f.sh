#!/bin/bash
# Full GPU suite; headline bench fp32 (tuned plans) / deterministic / bf16; rocprof kernel stats.
set -o pipefail
mkdir -p gpurun_out/prof_f32f
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  > gpurun_out/r3f_gputests.log 2>&1
rc=$?
tail -8 gpurun_out/r3f_gputests.log
# 1 = some tests failed (keep measuring); anything else (crash, timeout) stops the run
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 5 --warmup 1 > gpurun_out/r3f_bench_fp32.log 2>&1 || { tail -20 gpurun_out/r3f_bench_fp32.log; exit 1; }
tail -1 gpurun_out/r3f_bench_fp32.log
DDL_F32_MATH=x6 timeout -k 10 400 python -u bench.py --steps 5 --warmup 1 > gpurun_out/r3f_bench_x6.log 2>&1 || { tail -20 gpurun_out/r3f_bench_x6.log; exit 1; }
tail -1 gpurun_out/r3f_bench_x6.log
timeout -k 10 400 python -u scripts/conv_f32_tune.py --math x6 --out gpurun_out/f32_plans_x6_g8.json --groups 8 --budget-s 300 \
  > gpurun_out/r3f_tune_x6.log 2>&1 || { tail -5 gpurun_out/r3f_tune_x6.log; exit 1; }
tail -2 gpurun_out/r3f_tune_x6.log
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
PYTHONPATH=. timeout -k 10 200 python -u scripts/gemm_vs_blas.py > gpurun_out/r3f_gemm.log 2>&1 || { tail -20 gpurun_out/r3f_gemm.log; exit 1; }
cat gpurun_out/r3f_gemm.log
timeout -k 10 300 python -u benchmarks/bench_llm.py --steps 30 --warmup 5 > gpurun_out/r3f_llm.log 2>&1 || { tail -20 gpurun_out/r3f_llm.log; exit 1; }
tail -1 gpurun_out/r3f_llm.log
mkdir -p gpurun_out/prof_llm
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_llm -o run -- python -u benchmarks/bench_llm.py --steps 10 --warmup 3 \
  > gpurun_out/r3f_prof_llm.log 2>&1 || { tail -20 gpurun_out/r3f_prof_llm.log; exit 1; }
db=$(ls gpurun_out/prof_llm/*/run_results.db gpurun_out/prof_llm/run_results.db 2>/dev/null | head -n 1 || true)
[ -n "$db" ] && python scripts/prof_summary.py "$db" --top 40 > gpurun_out/r3f_prof_llm_summary.txt
timeout -k 10 300 python -u bench.py --steps 12 --warmup 1 --eval > gpurun_out/r3f_bench_eval.log 2>&1 || { tail -20 gpurun_out/r3f_bench_eval.log; exit 1; }
tail -1 gpurun_out/r3f_bench_eval.log
timeout -k 10 600 python -u benchmarks/bench_byzantine.py --steps 2 --warmup 1 --acc-rounds 8 > gpurun_out/r3f_byz.log 2>&1 || { tail -20 gpurun_out/r3f_byz.log; exit 1; }
tail -1 gpurun_out/r3f_byz.log
exit 0
