#!/bin/bash
# PMC passes of one halo-kernel launch (conv_x6h.hip): MFMA busy, waits, LDS, VALU.
#   bash scripts/gpu/pmc_x6h.sh <mode> <layer> [halo 0|1]
set -o pipefail
export TMPDIR=/tmp
O=$1; L=$2; H=${3:-1}; X=${4:-}
out=gpurun_out/pmcx/${O}_${L}_h${H}
mkdir -p $out
PA="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
PB="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAVES SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD"
i=0
for P in "$PA" "$PB"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P -d $out/p$i -o run -- python scripts/conv_f32_bench.py --math x6 --halo $H --mode $O --layer $L --reps 10 $X > $out/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $out/p$i.log; exit 1; }
done
tail -1 $out/p1.log
K=convx6h_kernel; [ "$H" = 0 ] && K=convf32_kernel
python scripts/pmc_dump.py $out $K
