#!/bin/bash
# RCCL world-1 + device pipeline tests; reference-equivalent eager baselines (fp32).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_rccl_pp_gpu.py -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r3_rccl_pp.log 2>&1
rc=$?
tail -8 gpurun_out/r3_rccl_pp.log
[ $rc -eq 0 ] || exit $rc
for v in faithful tuned_fp32 tuned; do
  timeout -k 10 600 python -u benchmarks/bench_reference_eager.py --variant $v --steps 1 --warmup 1 \
    >> gpurun_out/reference_eager_r3.jsonl 2> gpurun_out/r3_ref_$v.err || { tail -5 gpurun_out/r3_ref_$v.err; exit 1; }
  tail -1 gpurun_out/reference_eager_r3.jsonl
done
