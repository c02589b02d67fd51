#!/bin/bash
set -o pipefail
export PYTHONUNBUFFERED=1
run() { timeout -k 10 300 python -u benchmarks/bench_resnet50_dp.py --batch 256 --steps 5 --warmup 2 "$@" 2>&1 | grep '^{' | cut -c1-200; }
echo "default:"; run || exit 1
echo "bnfold off:"; DDL_F32_BNFOLD=0 run || exit 1
echo "64MB buckets:"; run --bucket-mb 64 || exit 1
