#!/bin/bash
# Memory-path PMC passes of one fp32 conv launch (L2 latency, L1 hits, TA/TCP stalls, LDS, VMEM levels).
#   bash scripts/gpu/pmc_f32_mem.sh <variant.so|default> <mode> <layer>
set -o pipefail
export TMPDIR=/tmp
LIB=$1; O=$2; L=$3
out=gpurun_out/pmcm/${O}_${L}
mkdir -p $out
[ "$LIB" != default ] && export DDL_KERNEL_LIB=$LIB
PA="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_VMEM_TA_ADDR_FIFO_FULL SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
PB="TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PERF_SEL_TOTAL_HIT_LRU_READ TCP_PERF_SEL_TOTAL_MISS_LRU_READ TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum SQ_WAIT_ANY SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS"
PC="TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_LFIFO_STALL_CYCLES_sum TCP_RFIFO_STALL_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TA_ADDR_STALLED_BY_TD_CYCLES_sum SQ_INSTS_VALU SQ_INSTS_SALU SQ_VALU_MFMA_COEXEC_CYCLES SQ_LDS_DATA_FIFO_FULL SQ_INST_LEVEL_LDS SQ_WAVES"
i=0
for P in "$PA" "$PB" "$PC"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P -d $out/p$i -o run -- python scripts/conv_f32_bench.py --math x6 --mode $O --layer $L --reps 10 > $out/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $out/p$i.log; exit 1; }
done
tail -1 $out/p1.log
python scripts/pmc_dump.py $out convf32_kernel
