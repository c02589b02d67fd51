#!/bin/bash
# PMC passes: halo vs streamed kernels on the layer-1 / layer-2 convs at 8 clients (heuristic
# selection, autotuner off). One counter group per run.
set -o pipefail
export TMPDIR=/tmp DDL_CONV_AUTOTUNE=0
out=gpurun_out/pmch2
mkdir -p $out
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES GRBM_GUI_ACTIVE"
P2="TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCC_EA0_RDREQ_sum"
for H in 1 0; do
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    DDL_CONV_HALO=$H timeout -s KILL 90 rocprofv3 --pmc $P -d $out/h${H}_p$i -o run -- python scripts/conv_bench.py --G 8 --layers c64,c128 > $out/h${H}_p$i.log 2>&1 || { echo "pmc $H $i failed"; tail -5 $out/h${H}_p$i.log; exit 1; }
  done
done
echo PMCOK
