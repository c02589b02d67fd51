#!/bin/bash
# halo numerics, halo sweep, then PMC: halo (auto) vs streamed on the layer-1 conv at 8 clients
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmch
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "halo or tile_configs" --timeout 120 --timeout-method thread > gpurun_out/th.log 2>&1; rc=$?; tail -3 gpurun_out/th.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/conv_bench.py --G 8 --sweep --layers c64,c128 > gpurun_out/hs8.log 2>&1 || exit 1
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES"
for H in 1 0; do
  DDL_CONV_HALO=$H timeout -s KILL 90 rocprofv3 --pmc $P1 -d gpurun_out/pmch/h$H -o run -- python scripts/conv_bench.py --G 8 --layers c64 > gpurun_out/pmch/h$H.log 2>&1 || { echo "pmc $H failed"; tail -5 gpurun_out/pmch/h$H.log; exit 1; }
done
echo PMCOK
