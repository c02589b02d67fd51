#!/bin/bash
# 1-client bench: halo split-K target A/B (DDL_F32_TARGET_WG; the halo plans' split-K heuristic)
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for TW in 640 400 256 1024; do
  r=$(DDL_F32_TARGET_WG=$TW timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --clients 1 --train-size 6250 2>&1 | tail -1 | cut -c1-120) || exit 1
  echo "TARGET_WG=$TW $r"
done
