#!/bin/bash
# gradient accuracy vs float64 torch for conv_x6h chain lengths 1 / 2 / 3 (3 = the default library)
set -o pipefail
export PYTHONUNBUFFERED=1
for V in 1 2 3; do for B in 16 50 100; do
  if [ $V != 3 ]; then export DDL_KERNEL_LIB=$PWD/ddl25spring_amd/lib/ab/libddl_kernels_ch$V.so; else unset DDL_KERNEL_LIB; fi
  echo "== chain $V batch $B"
  timeout -k 10 120 python scripts/debug_r18_grads.py --quiet --groups 1 --batch $B 2>&1 | grep -v amdgpu.ids | tail -3 | cut -c1-330 || exit 1
done; done
