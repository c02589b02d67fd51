#!/bin/bash
# nontemporal weight-image stores (abvar/splitnt.so) vs current: split kernel time + headline A/B
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for V in cur splitnt cur splitnt; do
  if [ $V = cur ]; then unset DDL_KERNEL_LIB; else export DDL_KERNEL_LIB=abvar/$V.so; fi
  echo "$V $(timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 2>&1 | tail -1 | cut -c95-140)" || exit 1
done
for V in cur splitnt; do
  if [ $V = cur ]; then unset DDL_KERNEL_LIB; else export DDL_KERNEL_LIB=abvar/$V.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5nt_$V -o run -- python bench.py --steps 1 --warmup 1 > gpurun_out/r5nt_$V.log 2>&1 || exit 1
  db=$(ls gpurun_out/r5nt_$V/*/run_results.db gpurun_out/r5nt_$V/run_results.db 2>/dev/null | head -1)
  echo "$V $(python scripts/prof_summary.py "$db" --top 60 | grep split_weights_multi)"
  rm -rf gpurun_out/r5nt_$V
done
