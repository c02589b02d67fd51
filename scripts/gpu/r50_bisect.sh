#!/bin/bash
# Bisect the ResNet-50 fp32 gradient mismatch over the WGRAD side stream and the engine choice.
set -o pipefail
mkdir -p gpurun_out
for cfg in "DDL_WGRAD_OVERLAP=0" "DDL_F32_MATH=mfma32" "DDL_WGRAD_OVERLAP=0 DDL_F32_MATH=mfma32" "DDL_F32_TUNED=0 DDL_WGRAD_OVERLAP=0"; do
  env $cfg timeout -k 10 300 python -u -m pytest tests/test_fp32_gpu.py -q -x -k "resnet50 and not mfma32 and not x6" --timeout 250 --timeout-method thread > gpurun_out/r50b.log 2>&1
  echo "== $cfg: $(tail -1 gpurun_out/r50b.log)"
  grep -o "ResNet-50 fp32 gradient errors:.*" gpurun_out/r50b.log | tr ' ' '\n' | grep "=" | awk -F= '$2 > 1e-4' | head -12 | tr '\n' ' '; echo
done
