#!/bin/bash
# round 5: halo WGRAD probes (device time) + 4x4 layer plans (old engine vs pinned halo kernel)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=${1:-r5j}
[ -n "$SKIP_HW" ] || T=${T}_hw PROBE_VAR=DDL_HW_PROBE KGREP=convx6hw CFGS="wgrad:c64 wgrad:c128" PROBES="0 1 2 4 3 5 6" \
  bash scripts/gpu/x6h_probe_trace.sh || exit 1
T=${T}_l4 KGREP="convx6h_kernel\|convf32_kernel" PROBES=0 CFGS="fwd:c512 fwd:c512:--pin,64/128/1/x6h fwd:c512:--pin,128/128/1/x6h fwd:c512:--pin,64/128/2/x6h dgrad:c512 dgrad:c512:--pin,64/128/1/x6h dgrad:c512:--pin,128/128/1/x6h dgrad:c512:--pin,64/128/2/x6h fwd:c256 fwd:c256:--pin,64/128/1/x6h" \
  bash scripts/gpu/x6h_probe_trace.sh
