#!/bin/bash
# Wave-cycle breakdown (waiting / issue-stalled / issuing, MFMA busy) of the conv kernels of one
# ResNet-18 layer, one PMC pass per counter group.
#   bash scripts/gpu/pmc_waits.sh "8 1" "c64 c512"
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/pmcw
mkdir -p $out
GS=${1:-"8 1"}
LS=${2:-"c64 c512"}
PA="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVES GRBM_GUI_ACTIVE"
PB="SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU"
for G in $GS; do
  for L in $LS; do
    i=0
    for P in "$PA" "$PB"; do
      i=$((i+1))
      timeout -s KILL 90 rocprofv3 --pmc $P -d $out/g${G}_${L}_p$i -o run -- python scripts/conv_bench.py --G $G --layers $L --epi > $out/g${G}_${L}_p$i.log 2>&1 || { echo "pass $G $L $i failed"; tail -5 $out/g${G}_${L}_p$i.log; exit 1; }
    done
  done
done
echo PMCDONE
