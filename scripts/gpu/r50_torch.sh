#!/bin/bash
# Stock PyTorch-ROCm fp32 ResNet-50 baseline with MIOpen's normal find (heartbeat keeps the run alive).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u benchmarks/bench_resnet50_torch.py --batch 256 --steps 8 --warmup 3 > gpurun_out/r50_torch.log 2>&1 || { tail -20 gpurun_out/r50_torch.log; exit 1; }
tail -1 gpurun_out/r50_torch.log | cut -c1-250
