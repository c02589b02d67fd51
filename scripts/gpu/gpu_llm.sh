#!/bin/bash
# LLaMA tutorial path: tests, tokens/s and a kernel profile.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_llama_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/tl.log 2>&1 && tail -2 gpurun_out/tl.log &&
timeout -k 10 300 python benchmarks/bench_llm.py --steps 20 --warmup 3 2>&1 | grep '^{' &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profllm -o run -- python benchmarks/bench_llm.py --steps 5 --warmup 2 > gpurun_out/profllm.log 2>&1 && echo PROFOK
