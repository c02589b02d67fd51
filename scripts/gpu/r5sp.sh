#!/bin/bash
# LDS-restaged weight-image stores: halo tests, split kernel time, headline
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_x6h_gpu.py > gpurun_out/r5sp_t.log 2>&1; rc=$?
tail -1 gpurun_out/r5sp_t.log; [ $rc = 0 ] || { grep -m5 "Error\|FAILED\|assert" gpurun_out/r5sp_t.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5sp_p -o run -- python bench.py --steps 1 --warmup 1 > gpurun_out/r5sp_p.log 2>&1 || exit 1
db=$(ls gpurun_out/r5sp_p/*/run_results.db gpurun_out/r5sp_p/run_results.db 2>/dev/null | head -1)
echo "$(python scripts/prof_summary.py "$db" --top 60 | grep split_weights_multi)"
rm -rf gpurun_out/r5sp_p
for r in 1 2; do echo "g8 $(timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 2>&1 | tail -1 | cut -c95-140)" || exit 1; done
echo "g1 $(timeout -k 10 300 python -u bench.py --clients 1 --train-size 6250 --steps 5 --warmup 2 2>&1 | tail -1 | cut -c95-140)"
