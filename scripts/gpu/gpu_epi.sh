#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python scripts/conv_bench.py --G 8 --sweep --epi --layers c64,c128,c256 > gpurun_out/he8.log 2>&1 &&
timeout -k 10 300 python scripts/conv_bench.py --G 1 --sweep --epi --layers c64,c128,c256 > gpurun_out/he1.log 2>&1 && echo EPIOK
