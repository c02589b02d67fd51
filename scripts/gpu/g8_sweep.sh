#!/bin/bash
set -o pipefail
export PYTHONUNBUFFERED=1
run() { timeout -k 10 200 python -u bench.py --steps 4 --warmup 2 2>&1 | grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"; }
for W in 256 384 640 1024; do echo "target_wg=$W: $(DDL_F32_TARGET_WG=$W run)" || exit 1; done
echo "wgrad overlap off: $(DDL_WGRAD_OVERLAP=0 run)"
