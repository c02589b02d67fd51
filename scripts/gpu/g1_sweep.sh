#!/bin/bash
set -o pipefail
export PYTHONUNBUFFERED=1
run() { timeout -k 10 200 python -u bench.py --clients 1 --train-size 6250 --steps 5 --warmup 2 2>&1 | grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"; }
for T in 1 0; do for W in 256 384 640 1024; do
  echo "tuned=$T target_wg=$W: $(DDL_F32_TUNED=$T DDL_F32_TARGET_WG=$W run)" || exit 1
done; done
