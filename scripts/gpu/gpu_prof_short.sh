#!/bin/bash
# Kernel-stats profile of the default headline bench; keeps only the summary CSVs (the raw trace exceeds gpurun's copy-back cap).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/final
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof -o run -- python3 bench.py --steps 20 --warmup 5 > gpurun_out/final/prof.log 2>&1 || { tail -20 gpurun_out/final/prof.log; exit 1; }
for f in $(find /tmp/prof -name "*stats.csv"); do cp "$f" gpurun_out/final/; done
grep '^{' gpurun_out/final/prof.log | cut -c1-200
ls gpurun_out/final
