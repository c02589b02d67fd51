#!/bin/bash
# The headline's old-engine WGRAD layers (8 clients): TF/s per layer, and one PMC pass on the 8x8 / c256 layer
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6w
for L in c256 c512 c128s2 sc128 c128 c64; do
  timeout -k 10 120 python -u scripts/conv_f32_bench.py --math auto --mode wgrad --G 8 --layer $L --reps 10 2>&1 | tail -1 || exit 1
done
PA="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
PB="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAVES SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD"
i=0
for P in "$PA" "$PB"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P -d gpurun_out/r6w/p$i -o run -- python scripts/conv_f32_bench.py --math auto --mode wgrad --G 8 --layer c256 --reps 5 > gpurun_out/r6w/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/r6w/p$i.log; exit 1; }
done
python scripts/pmc_dump.py gpurun_out/r6w convf32_kernel
