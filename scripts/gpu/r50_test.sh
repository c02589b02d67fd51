set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_fp32_gpu.py -q -x -k resnet50 --timeout 500 --timeout-method thread > gpurun_out/r50_test.log 2>&1; tail -12 gpurun_out/r50_test.log | cut -c1-3000
