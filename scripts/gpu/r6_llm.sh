#!/bin/bash
# round 6: planes-GEMM tests, fp32 LLaMA tests, bench_llm (native linears) and its kernel profile
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=${1:-r6l}
timeout -k 10 300 python -u -m pytest tests/test_gemm_x6_gpu.py tests/test_llama_f32_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${T}_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/${T}_tests.log | head -20; exit $rc; }
timeout -k 10 300 python -u benchmarks/bench_llm.py > gpurun_out/${T}_bench.log 2>&1 || { tail -20 gpurun_out/${T}_bench.log; exit 1; }
grep '^{' gpurun_out/${T}_bench.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${T} -o run -- python benchmarks/bench_llm.py --steps 5 --warmup 2 > gpurun_out/prof_${T}.log 2>&1 && echo PROFOK
