#!/bin/bash
# X6 ceiling probes: swizzle fix (sw), no operand split (nosplit), no IEEE adds (noadd), both.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for V in sw both noload nostore nobar noloadbar; do
  for L in c64 c256 c128s2; do for O in fwd dgrad wgrad; do
    echo -n "$V " >> gpurun_out/r3n_layers.log
    DDL_KERNEL_LIB=abvar/$V.so timeout -k 10 60 python scripts/conv_f32_bench.py --math x6 --mode $O --layer $L --reps 20 2>/dev/null >> gpurun_out/r3n_layers.log || { tail -5 gpurun_out/r3n_layers.log; exit 1; }
  done; done
done
cat gpurun_out/r3n_layers.log
