#!/bin/bash
# Last check of the final tree: the ResNet-50 fp32 test, smoke(), and a headline kernel profile.
set -o pipefail
mkdir -p gpurun_out/prof_last
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_fp32_gpu.py -q -x -k "resnet" --timeout 500 --timeout-method thread > gpurun_out/last_tests.log 2>&1 || { tail -30 gpurun_out/last_tests.log; exit 1; }
tail -1 gpurun_out/last_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/last_smoke.log 2>&1 || { tail -20 gpurun_out/last_smoke.log; exit 1; }
tail -1 gpurun_out/last_smoke.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_last -o run -- python -u bench.py --steps 3 --warmup 1 \
  > gpurun_out/last_prof.log 2>&1 || { tail -20 gpurun_out/last_prof.log; exit 1; }
db=$(ls gpurun_out/prof_last/*/run_results.db gpurun_out/prof_last/run_results.db 2>/dev/null | head -n 1 || true)
[ -n "$db" ] && python scripts/prof_summary.py "$db" --top 30 > gpurun_out/last_prof_summary.txt
head -8 gpurun_out/last_prof_summary.txt
