#!/bin/bash
# Round rehearsal: full GPU suite, smoke(), headline bench (default flags) and the deterministic bench.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/suite_gputests.log 2>&1
rc=$?
tail -6 gpurun_out/suite_gputests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/suite_smoke.log 2>&1 || { tail -20 gpurun_out/suite_smoke.log; exit 1; }
tail -1 gpurun_out/suite_smoke.log | cut -c1-300
timeout -k 10 300 python -u bench.py > gpurun_out/suite_bench_default.log 2>&1 || { tail -20 gpurun_out/suite_bench_default.log; exit 1; }
tail -1 gpurun_out/suite_bench_default.log
timeout -k 10 300 python -u bench.py --deterministic --steps 3 > gpurun_out/suite_bench_det.log 2>&1 || { tail -20 gpurun_out/suite_bench_det.log; exit 1; }
tail -1 gpurun_out/suite_bench_det.log
exit $rc
