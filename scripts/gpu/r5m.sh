#!/bin/bash
# WGRAD on 8x8 (c256) with the halo WGRAD allowed (HW_MIN_W 8) vs conv_f32
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=${1:-r5m}_w KGREP="convx6hw_kernel\|convf32_kernel<2" PROBES=0 CFGS="wgrad:c256 wgrad:c512" bash scripts/gpu/x6h_probe_trace.sh || exit 1
DDL_F32_HW_MIN_W=8 T=${1:-r5m}_w8 KGREP="convx6hw_kernel\|convf32_kernel<2" PROBES=0 CFGS="wgrad:c256" bash scripts/gpu/x6h_probe_trace.sh
