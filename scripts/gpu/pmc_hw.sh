#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/pmchw
mkdir -p $out
PA="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
PB="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_WAVES SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_LDS_IDX_ACTIVE"
i=0
for P in "$PA" "$PB"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P -d $out/p$i -o run -- python scripts/conv_f32_bench.py --math auto --mode wgrad --layer c128 --reps 10 > $out/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $out/p$i.log; }
done
python scripts/pmc_dump.py $out convx6hw
