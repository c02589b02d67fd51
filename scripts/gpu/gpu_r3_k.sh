#!/bin/bash
# 2-deep operand prefetch in conv_f32 + attention staging: fp32 + llama numerics, per-layer timing,
# headline bench (X6 default), LLM bench.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_fp32_gpu.py tests/test_llama_gpu.py -q --timeout 300 --timeout-method thread > gpurun_out/r3k_tests.log 2>&1
rc=$?
tail -4 gpurun_out/r3k_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for L in c64 c256 c512 c128s2; do for O in fwd dgrad wgrad; do for M in mfma32 x6; do
  timeout -k 10 60 python scripts/conv_f32_bench.py --math $M --mode $O --layer $L --reps 20 2>/dev/null >> gpurun_out/r3k_layers.log || { tail -5 gpurun_out/r3k_layers.log; exit 1; }
done; done; done
cat gpurun_out/r3k_layers.log
timeout -k 10 300 python -u bench.py --steps 5 > gpurun_out/r3k_bench.log 2>&1 || { tail -20 gpurun_out/r3k_bench.log; exit 1; }
tail -1 gpurun_out/r3k_bench.log
timeout -k 10 300 python -u benchmarks/bench_llm.py --steps 30 --warmup 5 > gpurun_out/r3k_llm.log 2>&1 || { tail -20 gpurun_out/r3k_llm.log; exit 1; }
tail -1 gpurun_out/r3k_llm.log
exit $rc
