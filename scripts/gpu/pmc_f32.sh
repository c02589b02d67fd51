#!/bin/bash
# PMC wave-cycle breakdown of the fp32 conv kernels (exact vs X6), one pass per counter group.
#   bash scripts/gpu/pmc_f32.sh "mfma32 x6" "fwd wgrad" "c64 c512"
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/pmcf
mkdir -p $out
MS=${1:-"mfma32 x6"}
MO=${2:-"fwd"}
LS=${3:-"c64"}
PA="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVES GRBM_GUI_ACTIVE"
PB="SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU"
PC="SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA TCC_HIT_sum TCC_MISS_sum"
for M in $MS; do
  for O in $MO; do
    for L in $LS; do
      i=0
      for P in "$PA" "$PB" "$PC"; do
        i=$((i+1))
        timeout -s KILL 90 rocprofv3 --pmc $P -d $out/${M}_${O}_${L}_p$i -o run -- python scripts/conv_f32_bench.py --math $M --mode $O --layer $L --reps 10 > $out/${M}_${O}_${L}_p$i.log 2>&1 || { echo "pass $M $O $L $i failed"; tail -5 $out/${M}_${O}_${L}_p$i.log; exit 1; }
      done
      tail -1 $out/${M}_${O}_${L}_p1.log
    done
  done
done
echo PMCDONE
