#!/bin/bash
# PMC wave-cycle breakdown of the fp32 attention kernels (one pass per counter group)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/pmca
mkdir -p $out
PA="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVES GRBM_GUI_ACTIVE"
PB="SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU"
i=0
for P in "$PA" "$PB"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P -d $out/attn_p$i -o run -- python scripts/attn_f32_bench.py --reps 5 > $out/attn_p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $out/attn_p$i.log; exit 1; }
done
echo PMCDONE
