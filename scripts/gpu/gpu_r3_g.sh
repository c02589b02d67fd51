#!/bin/bash
# fp32 conv PMC: exact vs X6 on the 32x32 / 4x4 3x3 layers (fwd, wgrad).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 bash scripts/gpu/pmc_f32.sh "mfma32 x6" "fwd wgrad" "c64 c512" > gpurun_out/r3g_pmc.log 2>&1
rc=$?
tail -12 gpurun_out/r3g_pmc.log
[ $rc -eq 0 ] || exit $rc
python scripts/pmc_waits_summary.py gpurun_out/pmcf convf32 > gpurun_out/r3g_pmc_summary.txt 2>&1
cat gpurun_out/r3g_pmc_summary.txt
