#!/bin/bash
# Round-3 fp32 bring-up on one MI355X: fp32 kernel numerics, smoke, a short headline bench.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_fp32_gpu.py -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r3_fp32_tests.log 2>&1
rc=$?
tail -40 gpurun_out/r3_fp32_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_smoke.log 2>&1 || { tail -30 gpurun_out/r3_smoke.log; exit 1; }
tail -3 gpurun_out/r3_smoke.log
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 > gpurun_out/r3_bench_fp32.log 2>&1
rc=$?
tail -5 gpurun_out/r3_bench_fp32.log
exit $rc
