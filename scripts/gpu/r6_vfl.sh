#!/bin/bash
# round 6: fused split-NN epoch kernel: numerics tests, config #5 bench (fused vs HIP-graph engine), rocprof
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=${1:-r6v}
timeout -k 10 300 python -u -m pytest tests/test_mlp_epoch_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${T}_tests.log; [ $rc -eq 0 ] || { grep -E "assert|Error|FAIL" gpurun_out/${T}_tests.log | head -20; exit $rc; }
cd benchmarks
timeout -k 10 300 python -u bench_vfl_gan.py --steps 20 --warmup 3 --gan-precisions fp32 --local-steps 2 > ../gpurun_out/${T}_bench_fused.log 2>&1 && grep '^{' ../gpurun_out/${T}_bench_fused.log | head -1
timeout -k 10 300 python -u bench_vfl_gan.py --steps 20 --warmup 3 --gan-precisions fp32 --local-steps 2 --vfl-engine graph > ../gpurun_out/${T}_bench_graph.log 2>&1 && grep '^{' ../gpurun_out/${T}_bench_graph.log | head -1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/${T}_prof -o prof -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_vfl_gan.py --steps 20 --warmup 3 --gan-precisions fp32 --local-steps 2 > $GRAFT_REPO_ROOT/gpurun_out/${T}_prof.log 2>&1
echo prof rc=$?
find $GRAFT_REPO_ROOT/gpurun_out/${T}_prof -name "*kernel_stats.csv" | head -2 | while read f; do head -12 "$f" | cut -c1-200; done
