#!/bin/bash
# round 5: bench + isolated step trace after the transposed halo epilogue
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=${1:-r5f}
step() {  # name timeout cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > gpurun_out/${T}_${name}.log 2>&1
  local rc=$?
  echo "[$name] rc=$rc :: $(tail -1 gpurun_out/${T}_${name}.log | cut -c1-400)"
  case $rc in 0) ;; *) echo "[$name] failed: stopping"; tail -30 gpurun_out/${T}_${name}.log; exit 1;; esac
}
step bench8 300 python -u bench.py --steps 5 --warmup 2
step bench1 300 python -u bench.py --steps 5 --warmup 2 --clients 1 --train-size 6250
export DDL_WGRAD_OVERLAP=0
step trace8 300 rocprofv3 --kernel-trace -d gpurun_out/${T}_trace8 -o run -- python bench.py --steps 1 --warmup 1
db=$(ls gpurun_out/${T}_trace8/*/run_results.db gpurun_out/${T}_trace8/run_results.db 2>/dev/null | head -1)
python scripts/step_trace_db.py "$db" > gpurun_out/${T}_step8.txt
python scripts/prof_summary.py "$db" --top 40 > gpurun_out/${T}_top8.txt
tail -1 gpurun_out/${T}_step8.txt
rm -rf gpurun_out/${T}_trace8
