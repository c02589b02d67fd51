#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
PT="python -u -X faulthandler -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu"
timeout -k 10 400 $PT tests/test_fl_gpu.py > gpurun_out/ah_fl.log 2>&1; rc=$?; echo "fl alone rc=$rc: $(tail -1 gpurun_out/ah_fl.log)"
case $rc in 124|137|139) exit $rc;; esac
timeout -k 10 400 $PT tests/test_dcgan.py tests/test_fl_gpu.py > gpurun_out/ah_both.log 2>&1; rc=$?; echo "dcgan+fl rc=$rc: $(tail -1 gpurun_out/ah_both.log)"
