#!/bin/bash
# Unsynchronised timed rounds: FL GPU tests, then 1 / 2 / 8-client bench A/B (--sync-rounds
# alternating) and the per-round idle time of the async mode from a kernel trace.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/async
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_fl_gpu.py tests/test_multirank_gpu.py -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
b() { local name=$1; shift; timeout -k 10 300 "$@" > $out/$name.log 2>&1 || { tail -5 $out/$name.log; exit 1; }; echo "$name: $(grep -o '"value": [0-9.]*' $out/$name.log)"; }
for rep in 1 2; do
  b c1_sync_$rep python bench.py --clients 1 --train-size 6250 --steps 6 --warmup 2 --sync-rounds
  b c1_async_$rep python bench.py --clients 1 --train-size 6250 --steps 6 --warmup 2
  b c8_sync_$rep python bench.py --steps 3 --warmup 1 --sync-rounds
  b c8_async_$rep python bench.py --steps 3 --warmup 1
done
b c2_sync python bench.py --clients 2 --train-size 12500 --steps 4 --warmup 1 --sync-rounds
b c2_async python bench.py --clients 2 --train-size 12500 --steps 4 --warmup 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/t -o run -- python bench.py --clients 1 --train-size 6250 --steps 4 --warmup 2 > $out/t.log 2>&1 || exit 1
f=$(find $out/t -name '*kernel_trace.csv' | head -1)
python scripts/round_gaps.py "$f" 5
rm -rf $out/t
