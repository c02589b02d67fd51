#!/bin/bash
# Short round-end rehearsal: GPU tests, smoke, default 1-GPU bench and a kernel-stats profile of it.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/final
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final/tests.log 2>&1 || { tail -30 gpurun_out/final/tests.log; exit 1; }
tail -1 gpurun_out/final/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || { tail -20 gpurun_out/final/smoke.log; exit 1; }
grep smoke gpurun_out/final/smoke.log | cut -c1-200
timeout -k 10 300 python bench.py > gpurun_out/final/bench_default.log 2>&1 || { tail -20 gpurun_out/final/bench_default.log; exit 1; }
grep '^{' gpurun_out/final/bench_default.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/final/prof -o run -- python3 bench.py --steps 20 --warmup 5 > gpurun_out/final/prof.log 2>&1 || { tail -20 gpurun_out/final/prof.log; exit 1; }
find gpurun_out/final/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/final/kernel_stats.csv
echo done
