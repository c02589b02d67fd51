#!/bin/bash
# the driver's round-end GPU tier: every @pytest.mark.gpu test, then smoke()
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/full_gpu.log 2>&1; rc=$?
tail -15 gpurun_out/full_gpu.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/full_smoke.log 2>&1; echo "smoke rc=$?"; tail -3 gpurun_out/full_smoke.log
