#!/bin/bash
# round 5: fp32 path checks after the bookkeeping changes, then 8- and 1-client bench + 1-client trace
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=${1:-r5b}
step() {  # name timeout cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > gpurun_out/${T}_${name}.log 2>&1
  local rc=$?
  echo "[$name] rc=$rc :: $(tail -1 gpurun_out/${T}_${name}.log | cut -c1-300)"
  case $rc in 0) ;; *) echo "[$name] failed: stopping"; tail -30 gpurun_out/${T}_${name}.log; exit 1;; esac
}
step tests 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_fp32_gpu.py tests/test_x6h_gpu.py
step bench8 300 python -u bench.py --steps 5 --warmup 2
step bench1 300 python -u bench.py --steps 5 --warmup 2 --clients 1 --train-size 6250
step trace1 300 rocprofv3 --kernel-trace -d gpurun_out/${T}_trace1 -o run -- python bench.py --steps 1 --warmup 1 --clients 1 --train-size 6250
db=$(ls gpurun_out/${T}_trace1/*/run_results.db gpurun_out/${T}_trace1/run_results.db 2>/dev/null | head -1)
python scripts/step_trace_db.py "$db" > gpurun_out/${T}_step1.txt
tail -1 gpurun_out/${T}_step1.txt
rm -rf gpurun_out/${T}_trace1
