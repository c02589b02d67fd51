#!/bin/bash
# chunked round graph: FL GPU tests, LLaMA fp32 tests (register CE), then the 500-step single-client round
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_fl_gpu.py tests/test_llama_f32_gpu.py > gpurun_out/r5z2_t.log 2>&1 || { tail -30 gpurun_out/r5z2_t.log; exit 1; }
tail -1 gpurun_out/r5z2_t.log
timeout -k 10 300 python -X faulthandler -u bench.py --clients 1 --steps 2 --warmup 1 > gpurun_out/r5z2_big.log 2>&1 || { tail -30 gpurun_out/r5z2_big.log; exit 1; }
tail -1 gpurun_out/r5z2_big.log | cut -c1-200
