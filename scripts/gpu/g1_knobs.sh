#!/bin/bash
# 1-client (per-GPU load of the 8-GPU headline) knob sweep: halo WGRAD on/off and its split target,
# conv_f32 split-K target
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
run() {  # label env...
  local label=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 5 --warmup 2 --clients 1 --train-size 6250 > gpurun_out/g1k.json 2> gpurun_out/g1k.err || { echo "$label failed"; tail -3 gpurun_out/g1k.err; exit 1; }
  echo "$label $(tail -1 gpurun_out/g1k.json | cut -c100-150)"
}
run default DDL_X=0
run hw_off DDL_F32_HALO_WGRAD=0
run hw_t512 DDL_F32_HW_TARGET_WG=512
run hw_t128 DDL_F32_HW_TARGET_WG=128
run tw1280 DDL_F32_TARGET_WG=1280
run tw320 DDL_F32_TARGET_WG=320
