#!/bin/bash
# Full GPU suite with X6 as the default fp32 engine; smoke; headline bench (default flags).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r3j_gputests.log 2>&1
rc=$?
tail -6 gpurun_out/r3j_gputests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3j_smoke.log 2>&1 || { tail -20 gpurun_out/r3j_smoke.log; exit 1; }
tail -1 gpurun_out/r3j_smoke.log | cut -c1-300
timeout -k 10 300 python -u bench.py > gpurun_out/r3j_bench_default.log 2>&1 || { tail -20 gpurun_out/r3j_bench_default.log; exit 1; }
tail -1 gpurun_out/r3j_bench_default.log
timeout -k 10 300 python -u bench.py --deterministic --steps 3 > gpurun_out/r3j_bench_det.log 2>&1 || { tail -20 gpurun_out/r3j_bench_det.log; exit 1; }
tail -1 gpurun_out/r3j_bench_det.log
exit $rc
