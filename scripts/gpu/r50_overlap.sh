#!/bin/bash
# ResNet-50 DP at world 1 over a forced RCCL process group (DDL_FORCE_PG=1): the bucketed
# all-reduces are real RCCL launches, so a kernel trace shows whether they run concurrently with
# the later layers' backward kernels. Writes gpurun_out/r50_overlap.txt.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp DDL_FORCE_PG=1 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29871
B=${1:-128}
timeout -k 10 300 python -u benchmarks/bench_resnet50_dp.py --batch $B --steps 5 --warmup 2 > gpurun_out/r50_bench.log 2>&1 || { tail -20 gpurun_out/r50_bench.log; exit 1; }
tail -1 gpurun_out/r50_bench.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r50_prof -o run -- python benchmarks/bench_resnet50_dp.py --batch $B --steps 2 --warmup 1 > gpurun_out/r50_prof.log 2>&1 || { tail -20 gpurun_out/r50_prof.log; exit 1; }
DB=$(ls gpurun_out/r50_prof/*/run_results.db gpurun_out/r50_prof/run_results.db 2>/dev/null | head -1)
python scripts/overlap_report.py $DB > gpurun_out/r50_overlap.txt
python scripts/prof_summary.py $DB --top 25 >> gpurun_out/r50_overlap.txt
tail -40 gpurun_out/r50_overlap.txt
