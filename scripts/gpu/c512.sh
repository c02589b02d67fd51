#!/bin/bash
# c512 (4x4 images): halo FWD / DGRAD (3-step chains) vs conv_f32, per layer and in the headline
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for M in fwd dgrad; do for W in 8 4; do
  DDL_F32_HALO_MIN_W=$W timeout -k 10 60 python scripts/conv_f32_bench.py --math auto --mode $M --layer c512 --reps 20 2>&1 | tail -1 | sed "s/^/minw=$W /" || exit 1
done; done
for W in 8 4 8 4; do
  DDL_F32_HALO_MIN_W=$W timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_minw$W.json 2> gpurun_out/bench_minw$W.err || exit 1
  echo "minw=$W $(tail -1 gpurun_out/bench_minw$W.json | cut -c100-160)"
done
