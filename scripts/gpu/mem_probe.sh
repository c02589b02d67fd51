#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for C in 1 8; do for O in 1 0; do
  DDL_WGRAD_OVERLAP=$O timeout -k 10 300 python -u scripts/mem_probe.py $C > gpurun_out/mem_${C}_$O.log 2>&1 || { tail -5 gpurun_out/mem_${C}_$O.log; exit 1; }
  tail -1 gpurun_out/mem_${C}_$O.log
done; done
