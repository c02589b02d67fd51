#!/bin/bash
# Round-4 measurement sweep: numerics after the packed split, then every secondary benchmark line
# (LLaMA fp32/bf16, MnistCnn fp32/bf16, Byzantine, DCGAN/VFL, 1-client headline, ResNet-50 DP +
# RCCL overlap trace). Results land in gpurun_out/r4f_*.log.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=r4f
step() {  # name timeout cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > gpurun_out/${T}_${name}.log 2>&1
  local rc=$?
  echo "[$name] rc=$rc :: $(grep -E '^\{|passed|failed' gpurun_out/${T}_${name}.log | tail -2 | cut -c1-400)"
  case $rc in 124|134|137|139) echo "[$name] crashed or timed out: stopping"; exit $rc;; esac
  return 0
}
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
step tests 600 $PT tests/test_x6h_gpu.py tests/test_fp32_gpu.py tests/test_llama_f32_gpu.py
step bench 300 python -u bench.py --steps 5 --warmup 2
step bench_c1 300 python -u bench.py --clients 1 --train-size 6250 --steps 5 --warmup 2
step llm 400 python -u benchmarks/bench_llm.py --steps 10 --warmup 3
step mnist 300 python -u benchmarks/bench_mnist_fedavg.py
step mnist_bf16 300 python -u benchmarks/bench_mnist_fedavg.py --precision bf16
step byz 600 python -u benchmarks/bench_byzantine.py --no-eval
step gan 300 python -u benchmarks/bench_vfl_gan.py
step gantest 300 $PT tests/test_dcgan.py tests/test_graphs_gpu.py -k "gan"
step prof_c1 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_c1 -o run -- python bench.py --clients 1 --train-size 6250 --steps 2 --warmup 1
python scripts/prof_summary.py $(ls gpurun_out/${T}_prof_c1/*/run_results.db gpurun_out/${T}_prof_c1/run_results.db 2>/dev/null | head -1) --top 30 > gpurun_out/${T}_prof_c1_summary.txt
head -30 gpurun_out/${T}_prof_c1_summary.txt
