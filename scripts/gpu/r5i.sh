#!/bin/bash
# round 5: fp32 tests after the epilogue rewrites + bench 8/1 clients + step traces at 8 and 1 client
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=${1:-r5i}
step() {  # name timeout cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > gpurun_out/${T}_${name}.log 2>&1
  local rc=$?
  echo "[$name] rc=$rc :: $(tail -1 gpurun_out/${T}_${name}.log | cut -c1-300)"
  case $rc in 0) ;; *) echo "[$name] failed: stopping"; tail -30 gpurun_out/${T}_${name}.log; exit 1;; esac
}
trace() {  # name clients
  local name=$1 C=$2
  step $name 300 rocprofv3 --kernel-trace -d gpurun_out/${T}_$name -o run -- python bench.py --steps 1 --warmup 1 --clients $C --train-size $((6250 * C))
  local db=$(ls gpurun_out/${T}_$name/*/run_results.db gpurun_out/${T}_$name/run_results.db 2>/dev/null | head -1)
  python scripts/step_trace_db.py "$db" > gpurun_out/${T}_${name}_step.txt
  python scripts/prof_summary.py "$db" --top 45 > gpurun_out/${T}_${name}_top.txt
  tail -1 gpurun_out/${T}_${name}_step.txt
  rm -rf gpurun_out/${T}_$name
}
step tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_fp32_gpu.py tests/test_x6h_gpu.py tests/test_fl_gpu.py
step bench8 300 python -u bench.py --steps 5 --warmup 2
step bench1 300 python -u bench.py --steps 5 --warmup 2 --clients 1 --train-size 6250
trace trace1 1
export DDL_WGRAD_OVERLAP=0
trace trace8 8
