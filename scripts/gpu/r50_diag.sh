#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u scratch/r50_diag.py > gpurun_out/r50_diag.log 2>&1; cat gpurun_out/r50_diag.log | grep -v amdgpu.ids
