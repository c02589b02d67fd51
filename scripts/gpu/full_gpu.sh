#!/bin/bash
# every @pytest.mark.gpu test
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/full_gpu.log 2>&1; rc=$?
tail -15 gpurun_out/full_gpu.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 5 30 ./scripts/lds_unaligned.bin || true
