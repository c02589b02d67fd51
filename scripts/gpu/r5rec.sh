#!/bin/bash
# record-and-tune the fp32 conv launches of the headline (8 and 1 clients) and the MnistCnn bench
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
val() { grep '^{' "$1" | tail -1 | grep -o '"value": [0-9.]*'; }
work() {  # tag cmd...
  local tag=$1; shift
  DDL_F32_RECORD=$PWD/gpurun_out/rec_$tag.json timeout -k 10 300 "$@" > gpurun_out/rec_${tag}_0.log 2>&1 || { tail -5 gpurun_out/rec_${tag}_0.log; exit 1; }
  echo "$tag before $(val gpurun_out/rec_${tag}_0.log)"
  timeout -k 10 600 python -u scripts/conv_f32_tune.py --geoms-file gpurun_out/rec_$tag.json --math auto --skip-halo --budget-s 400 --out gpurun_out/rec_${tag}_plans.json > gpurun_out/rec_${tag}_tune.log 2>&1 || { tail -5 gpurun_out/rec_${tag}_tune.log; exit 1; }
  cp ddl25spring_amd/ops/f32_plans.json gpurun_out/f32_plans_pre_$tag.json
  python scripts/merge_plans.py gpurun_out/rec_${tag}_plans.json
  timeout -k 10 300 "$@" > gpurun_out/rec_${tag}_1.log 2>&1 || { tail -5 gpurun_out/rec_${tag}_1.log; exit 1; }
  echo "$tag after $(val gpurun_out/rec_${tag}_1.log)"
  timeout -k 10 300 "$@" > gpurun_out/rec_${tag}_1.log 2>&1 || { tail -5 gpurun_out/rec_${tag}_1.log; exit 1; }
  echo "$tag after $(val gpurun_out/rec_${tag}_1.log)"
  cp ddl25spring_amd/ops/f32_plans.json gpurun_out/f32_plans_post_$tag.json
}
work g8 python -u bench.py --steps 5 --warmup 2
work g1 python -u bench.py --clients 1 --train-size 6250 --steps 5 --warmup 2
work mnist python -u benchmarks/bench_mnist_fedavg.py
