#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -v -k "wgrad" --timeout 120 --timeout-method thread > gpurun_out/tw.log 2>&1; rc=$?; grep -E "PASS|FAIL|Error|error" gpurun_out/tw.log | head -20; [ $rc -eq 0 ] || { tail -30 gpurun_out/tw.log; exit $rc; }
timeout -k 10 300 python scripts/conv_bench.py --G 8 --layers c64,c128,c256 --wh-splits 4,8,16,32,64 > gpurun_out/wh8.log 2>&1 && grep -v amdgpu.ids gpurun_out/wh8.log &&
timeout -k 10 300 python scripts/conv_bench.py --G 1 --layers c64,c128,c256 --wh-splits 2,4,8,16,32 > gpurun_out/wh1.log 2>&1 && grep -v amdgpu.ids gpurun_out/wh1.log
