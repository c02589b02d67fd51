#!/bin/bash
# Round-3 final rehearsal (full GPU suite, smoke, headline + deterministic benches), then the stock-torch
# fp32 ResNet-50 baseline (last: MIOpen's kernel search may run long).
set -o pipefail
bash scripts/gpu/gpu_suite.sh || exit $?
bash scripts/gpu/r50_torch.sh
