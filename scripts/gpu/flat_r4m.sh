#!/bin/bash
# which of FWD / DGRAD / WGRAD gains or loses from the 128-pixel-row 1x1 geometry (ResNet-50 fp32)
set -o pipefail
export PYTHONUNBUFFERED=1
run() { timeout -k 10 300 python -u benchmarks/bench_resnet50_dp.py --batch 256 --steps 5 --warmup 2 "$@" 2>&1 | grep '^{' | python3 -c "import json,sys; print(json.loads(sys.stdin.read())[\"value\"])"; }
for F in 0 w f d w 0; do echo "flat=$F $(DDL_F32_FLAT1X1=$F run)" || exit 1; done
