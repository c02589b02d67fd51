#!/bin/bash
# Generic iteration: all GPU tests, then the headline bench at 8 and 1 clients.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tg.log 2>&1; rc=$?; tail -3 gpurun_out/tg.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 3 --warmup 1 > gpurun_out/hb8.log 2>&1 && grep '^{' gpurun_out/hb8.log | cut -c1-200 &&
timeout -k 10 200 python bench.py --clients 1 --train-size 6250 --steps 3 --warmup 1 > gpurun_out/hb1.log 2>&1 && grep '^{' gpurun_out/hb1.log | cut -c1-200
