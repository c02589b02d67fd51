#!/bin/bash
# round 6: GEMM tests + microbench, IPC tests (ordered FedAvg mean), LLaMA fp32 tests
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=${1:-r6m}
timeout -k 10 800 python -u -m pytest tests/test_gemm_x6_gpu.py tests/test_ipc_gpu.py tests/test_llama_f32_gpu.py tests/test_fl_gpu.py tests/test_multirank_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_tests.log 2>&1
rc=$?; tail -2 gpurun_out/${T}_tests.log; [ $rc -eq 0 ] || { grep -E "assert|Error|FAIL" gpurun_out/${T}_tests.log | head -20; exit $rc; }
timeout -k 10 100 python -u scripts/gemm_x6_probe4.py 2>&1 | grep "^{" | cut -c1-120
timeout -k 10 200 python -u scripts/gemm_x6_bench.py > gpurun_out/${T}_gemm.jsonl 2>gpurun_out/${T}_gemm.err; cut -c1-160 gpurun_out/${T}_gemm.jsonl
