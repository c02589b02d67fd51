#!/bin/bash
# BN backward fold slot-block size A/B (FB_SB 64 = current, 32, 128) at 1 and 8 clients
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
for C in 1 8; do for V in cur fb32 fb128 cur fb32 fb128; do
  if [ $V = cur ]; then unset DDL_KERNEL_LIB; else export DDL_KERNEL_LIB=abvar/$V.so; fi
  echo "clients=$C $V $(timeout -k 10 300 python -u bench.py --clients $C --train-size $((6250 * C)) --steps 5 --warmup 2 2>&1 | tail -1 | cut -c95-140)" || exit 1
done; done
