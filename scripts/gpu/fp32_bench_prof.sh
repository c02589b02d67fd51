#!/bin/bash
# fp32 numerics (all fp32 GPU tests), the headline bench, and a kernel-trace profile of 2 rounds.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=${1:-r4}
timeout -k 10 600 python -u -m pytest tests/test_fp32_gpu.py tests/test_x6h_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_fp32_tests.log 2>&1 || { tail -40 gpurun_out/${T}_fp32_tests.log; exit 1; }
tail -1 gpurun_out/${T}_fp32_tests.log
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/${T}_bench.log 2>&1 || { tail -30 gpurun_out/${T}_bench.log; exit 1; }
tail -1 gpurun_out/${T}_bench.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run -- python bench.py --steps 2 --warmup 1 > gpurun_out/${T}_prof.log 2>&1 || { tail -20 gpurun_out/${T}_prof.log; exit 1; }
python scripts/prof_summary.py $(ls gpurun_out/${T}_prof/*/run_results.db gpurun_out/${T}_prof/run_results.db 2>/dev/null | head -1) --top 30 > gpurun_out/${T}_prof_summary.txt; cat gpurun_out/${T}_prof_summary.txt
