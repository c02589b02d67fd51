#!/bin/bash
# round 5: isolated per-kernel step trace (no WGRAD side stream) at 8 clients + PMC passes of the
# halo FWD (c128) and DGRAD (c64, BN-fold operand) kernels
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=${1:-r5d}
step() {  # name timeout cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > gpurun_out/${T}_${name}.log 2>&1
  local rc=$?
  echo "[$name] rc=$rc :: $(tail -1 gpurun_out/${T}_${name}.log | cut -c1-300)"
  case $rc in 0) ;; *) echo "[$name] failed: stopping"; tail -30 gpurun_out/${T}_${name}.log; exit 1;; esac
}
export DDL_WGRAD_OVERLAP=0
step bench8 300 python -u bench.py --steps 5 --warmup 2
step trace8 300 rocprofv3 --kernel-trace -d gpurun_out/${T}_trace8 -o run -- python bench.py --steps 1 --warmup 1
db=$(ls gpurun_out/${T}_trace8/*/run_results.db gpurun_out/${T}_trace8/run_results.db 2>/dev/null | head -1)
python scripts/step_trace_db.py "$db" > gpurun_out/${T}_step8.txt
tail -1 gpurun_out/${T}_step8.txt
rm -rf gpurun_out/${T}_trace8
unset DDL_WGRAD_OVERLAP
bash scripts/gpu/pmc_x6h.sh fwd c128 1 > gpurun_out/${T}_pmc_fwd_c128.txt 2>&1 || exit 1
cat gpurun_out/${T}_pmc_fwd_c128.txt | tail -22
bash scripts/gpu/pmc_x6h.sh dgrad c64 1 "--dybn 2" > gpurun_out/${T}_pmc_dgrad_c64.txt 2>&1 || exit 1
cat gpurun_out/${T}_pmc_dgrad_c64.txt | tail -22
step diag_sync4 300 python -u scripts/fl_sync_diag.py --reps 4 --modes sync
step diag_notune 300 env DDL_CONV_AUTOTUNE=0 python -u scripts/fl_sync_diag.py --reps 2 --modes sync,unsync,sync
step llm_flat 300 env DDL_F32_FLAT1X1=1 python -u benchmarks/bench_llm.py --precision fp32 --steps 10 --warmup 3
step llm_base 300 python -u benchmarks/bench_llm.py --precision fp32 --steps 10 --warmup 3
