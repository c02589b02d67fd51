#!/bin/bash
# round 5: halo-kernel timing probes (DDL_X6H_PROBE: 1 no weight DMA, 2 no halo loads, 4 no MFMAs;
# results WRONG, timing only), bf16 unsync diagnosis variants, LLM fp32 test after rmsf_fold change
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=${1:-r5e}
step() {  # name timeout cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > gpurun_out/${T}_${name}.log 2>&1
  local rc=$?
  echo "[$name] rc=$rc :: $(tail -1 gpurun_out/${T}_${name}.log | cut -c1-300)"
  case $rc in 0) ;; *) echo "[$name] failed: stopping"; tail -30 gpurun_out/${T}_${name}.log; exit 1;; esac
}
step llama 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_llama_f32_gpu.py
for cfg in "fwd c128" "fwd c64" "dgrad c64"; do
  set -- $cfg
  for p in 0 1 2 4 3 6 7; do
    step probe_${1}_${2}_$p 120 env DDL_X6H_PROBE=$p python -u scripts/conv_f32_bench.py --mode $1 --layer $2 --G 8 --reps 20
  done
done
export DDL_CONV_AUTOTUNE=0
step diag_modes 300 python -u scripts/fl_sync_diag.py --reps 2 --modes sync,unsync,unsync_s,sync
step diag_noovl 300 env DDL_WGRAD_OVERLAP=0 python -u scripts/fl_sync_diag.py --reps 1 --modes sync,unsync,sync
step diag_nodirect 300 env DDL_DIRECT_SGD=0 python -u scripts/fl_sync_diag.py --reps 1 --modes sync,unsync,sync
step diag_graphs2 300 env DDL_ROUND_GRAPHS=2 python -u scripts/fl_sync_diag.py --reps 1 --modes sync,unsync,sync
