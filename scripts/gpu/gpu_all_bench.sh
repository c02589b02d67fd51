#!/bin/bash
# Every BASELINE.json config's benchmark on one GPU (one JSON line each) + the headline profile.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/allbench
mkdir -p $out
run() { local name=$1 secs=$2; shift 2; timeout -k 10 $secs "$@" > $out/$name.log 2>&1; local rc=$?; grep '^{' $out/$name.log; [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -5 $out/$name.log; exit $rc; }; }
run headline8 300 python bench.py --steps 3 --warmup 1
run headline1 300 python bench.py --clients 1 --train-size 6250 --steps 3 --warmup 1
run mnist 300 python benchmarks/bench_mnist_fedavg.py --steps 20 --warmup 2
run resnet50 300 python benchmarks/bench_resnet50_dp.py --steps 10 --warmup 3
run llm 300 python benchmarks/bench_llm.py --steps 20 --warmup 3
run vflgan 300 python benchmarks/bench_vfl_gan.py
run byz 300 python benchmarks/bench_byzantine.py
run prof8 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof8 -o run -- python bench.py --steps 2 --warmup 1
run prof1 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof1 -o run -- python bench.py --clients 1 --train-size 6250 --steps 3 --warmup 1
# keep the kernel statistics and their summaries; the per-dispatch traces would overflow gpurun_out
for p in prof8 prof1; do
  f=$(find $out/$p -name '*kernel_stats.csv' | head -1)
  [ -n "$f" ] && python scripts/prof_summary.py "$f" 30 > $out/${p}_summary.txt && cp "$f" $out/${p}_kernel_stats.csv
  rm -rf $out/$p
done
echo ALLDONE
