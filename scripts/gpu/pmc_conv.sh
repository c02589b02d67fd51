#!/bin/bash
# PMC passes over the conv microbenchmark (one pass per counter group, each its own short run).
#   bash scripts/gpu/pmc_conv.sh "8 1" "c64 c256"
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/pmc
mkdir -p $out
GS=${1:-"8 1"}
LS=${2:-"c64 c256"}
P1="GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
P2="TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"
P3="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TA_BUSY_sum TD_BUSY_sum"
for G in $GS; do
  for L in $LS; do
    i=0
    for P in "$P1" "$P2" "$P3"; do
      i=$((i+1))
      timeout -s KILL 90 rocprofv3 --pmc $P -d $out/g${G}_${L}_p$i -o run -- python scripts/conv_bench.py --G $G --layers $L > $out/g${G}_${L}_p$i.log 2>&1 || { echo "pass $G $L $i failed"; tail -5 $out/g${G}_${L}_p$i.log; exit 1; }
    done
  done
done
echo PMCDONE
