#!/bin/bash
# round 6: every benchmark once, JSON lines collected in gpurun_out/${T}.jsonl
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=${1:-final_r6}
out=gpurun_out/${T}.jsonl
: > $out
run() {  # tag timeout cmd...
  local tag=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > gpurun_out/${T}_${tag}.log 2>&1
  local rc=$?
  echo "# $tag rc=$rc" >> $out
  grep '^{' gpurun_out/${T}_${tag}.log >> $out
  echo "[$tag] rc=$rc $(grep '^{' gpurun_out/${T}_${tag}.log | tail -1 | cut -c1-150)"
  case $rc in 0) ;; *) echo "[$tag] failed"; tail -20 gpurun_out/${T}_${tag}.log; exit 1;; esac
}
run bench8 300 python -u bench.py --steps 5 --warmup 2
for C in 4 2 1; do run bench_c$C 300 python -u bench.py --steps 5 --warmup 2 --clients $C --train-size $((6250 * C)); done
run bench_bf16 300 python -u bench.py --steps 5 --warmup 2 --precision bf16
run mnist 300 python -u benchmarks/bench_mnist_fedavg.py
run gan 300 python -u benchmarks/bench_vfl_gan.py
run llm 400 python -u benchmarks/bench_llm.py
run r50 400 python -u benchmarks/bench_resnet50_dp.py --steps 6 --warmup 3
run byz 400 python -u benchmarks/bench_byzantine.py
