#!/bin/bash
# round 6: X6 GEMM correctness + timing vs the vendor fp32 GEMM on the LLaMA linear shapes
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=${1:-r6g}
timeout -k 10 240 python -u scripts/gemm_x6_bench.py --check ${2:+--plans "$2"} > gpurun_out/${T}.jsonl 2> gpurun_out/${T}.err
rc=$?
cat gpurun_out/${T}.jsonl | cut -c1-260
tail -5 gpurun_out/${T}.err
exit $rc
