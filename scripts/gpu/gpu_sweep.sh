set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python scripts/conv_bench.py --G 8 --sweep > gpurun_out/sweep8.log 2>&1 && timeout -k 10 500 python scripts/conv_bench.py --G 1 --sweep > gpurun_out/sweep1.log 2>&1 && echo SWEEPOK
