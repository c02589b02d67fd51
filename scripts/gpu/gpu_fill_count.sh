#!/bin/bash
# Steady-state per-round kernel counts: kernel stats at two step counts; the difference / 20 is per timed round.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/fill
for s in 10 30; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/p$s -o run -- python3 bench.py --steps $s --warmup 5 > gpurun_out/fill/prof$s.log 2>&1 || { tail -20 gpurun_out/fill/prof$s.log; exit 1; }
  cp $(find /tmp/p$s -name "*kernel_stats.csv") gpurun_out/fill/kstats_$s.csv || exit 1
done
echo done
