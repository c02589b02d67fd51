#!/bin/bash
# round 5: row-padded halo widths (ResNet-50 56 / 28): tests, then the ResNet-50 DP bench with and
# without them, and a kernel trace of the padded run
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=${1:-r5p}
step() {  # name timeout cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > gpurun_out/${T}_${name}.log 2>&1
  local rc=$?
  echo "[$name] rc=$rc :: $(tail -1 gpurun_out/${T}_${name}.log | cut -c1-260)"
  case $rc in 0) ;; *) echo "[$name] failed: stopping"; tail -30 gpurun_out/${T}_${name}.log; exit 1;; esac
}
[ -n "$NOTEST" ] || step tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_x6h_gpu.py tests/test_fp32_gpu.py
step r50_nopadw 400 env DDL_F32_HALO_PADW=0 python -u benchmarks/bench_resnet50_dp.py --steps 6 --warmup 3
step r50_padw 400 python -u benchmarks/bench_resnet50_dp.py --steps 6 --warmup 3
for V in nopadw padw; do
E=""; [ $V = nopadw ] && E="DDL_F32_HALO_PADW=0"
step r50_trace_$V 400 env $E rocprofv3 --kernel-trace -d gpurun_out/${T}_r50tr_$V -o run -- python benchmarks/bench_resnet50_dp.py --steps 2 --warmup 2
db=$(ls gpurun_out/${T}_r50tr_$V/*/run_results.db gpurun_out/${T}_r50tr_$V/run_results.db 2>/dev/null | head -1)
python scripts/prof_summary.py "$db" --top 40 > gpurun_out/${T}_r50_top_$V.txt
head -3 gpurun_out/${T}_r50_top_$V.txt
rm -rf gpurun_out/${T}_r50tr_$V
done
