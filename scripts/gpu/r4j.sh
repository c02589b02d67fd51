#!/bin/bash
# round-4 late numbers: headline bench + rocprof summary, clients-per-GPU sweep
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=${1:-r4j}
step() {  # name timeout cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > gpurun_out/${T}_${name}.log 2>&1
  local rc=$?
  echo "[$name] rc=$rc :: $(tail -1 gpurun_out/${T}_${name}.log | cut -c1-260)"
  case $rc in 0) ;; *) echo "[$name] failed: stopping"; exit 1;; esac
}
for M in fwd dgrad; do for W in 8 4; do
  DDL_F32_HALO_MIN_W=$W timeout -k 10 60 python scripts/conv_f32_bench.py --math auto --mode $M --layer c512 --reps 20 2>&1 | tail -1 | sed "s/^/minw=$W /" || exit 1
done; done
step bench 300 python -u bench.py --steps 5 --warmup 2
for C in 1 2 4; do
  step clients$C 300 python -u bench.py --steps 5 --warmup 2 --clients $C --train-size $((6250 * C))
done
step prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run -- python bench.py --steps 2 --warmup 1
python scripts/prof_summary.py $(ls gpurun_out/${T}_prof/*/run_results.db gpurun_out/${T}_prof/run_results.db 2>/dev/null | head -1) --top 30 > gpurun_out/${T}_prof_summary.txt
head -24 gpurun_out/${T}_prof_summary.txt
step prof1 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof1 -o run -- python bench.py --steps 2 --warmup 1 --clients 1 --train-size 6250
python scripts/prof_summary.py $(ls gpurun_out/${T}_prof1/*/run_results.db gpurun_out/${T}_prof1/run_results.db 2>/dev/null | head -1) --top 30 > gpurun_out/${T}_prof1_summary.txt
head -16 gpurun_out/${T}_prof1_summary.txt
