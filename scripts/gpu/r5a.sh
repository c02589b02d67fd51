#!/bin/bash
# round-5 baseline: headline bench, then one traced local step per client count (kernel sequence)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=${1:-r5a}
step() {  # name timeout cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > gpurun_out/${T}_${name}.log 2>&1
  local rc=$?
  echo "[$name] rc=$rc :: $(tail -1 gpurun_out/${T}_${name}.log | cut -c1-300)"
  case $rc in 0) ;; *) echo "[$name] failed: stopping"; exit 1;; esac
}
step bench 300 python -u bench.py --steps 5 --warmup 2
for C in 8 1; do
  step trace$C 300 rocprofv3 --kernel-trace -d gpurun_out/${T}_trace$C -o run -- python bench.py --steps 1 --warmup 1 --clients $C --train-size $((6250 * C))
  db=$(ls gpurun_out/${T}_trace$C/*/run_results.db gpurun_out/${T}_trace$C/run_results.db 2>/dev/null | head -1)
  python scripts/step_trace_db.py "$db" > gpurun_out/${T}_step$C.txt
  tail -1 gpurun_out/${T}_step$C.txt
  rm -rf gpurun_out/${T}_trace$C
done
