set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_x6h_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/x6h_net_tests.log 2>&1 || { tail -60 gpurun_out/x6h_net_tests.log; exit 1; }
tail -1 gpurun_out/x6h_net_tests.log
timeout -k 10 400 python -u -m pytest tests/test_fp32_gpu.py -x -q --timeout 300 --timeout-method thread -k "resnet18" > gpurun_out/x6h_net_r18.log 2>&1 || { tail -40 gpurun_out/x6h_net_r18.log; exit 1; }
tail -1 gpurun_out/x6h_net_r18.log
