#!/bin/bash
# PMC passes of the conv_f32 WGRAD (what bounds it: MFMA busy, waits, L2 traffic)
#   bash scripts/gpu/pmc_wgrad.sh <layer>
set -o pipefail
export TMPDIR=/tmp
L=$1
out=gpurun_out/pmcw/$L
mkdir -p $out
PA="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
PB="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAVES SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD"
PC="TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum"
i=0
for P in "$PA" "$PB" "$PC"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P -d $out/p$i -o run -- python scripts/conv_f32_bench.py --math x6 --mode wgrad --layer $L --reps 10 > $out/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $out/p$i.log; }
done
tail -1 $out/p1.log
python scripts/pmc_dump.py $out convf32_kernel
