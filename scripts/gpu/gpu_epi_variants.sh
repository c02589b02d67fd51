#!/bin/bash
# Split-K epilogue variants (DDL_SPLITK_EPI = rows-per-thread x slices-per-round-trip): 1-client
# bench + rocprof kernel stats of the epilogue and conv launches per variant.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/epi
mkdir -p $out
DDL_TUNE_DEEP=0 timeout -k 10 300 python bench.py --clients 1 --train-size 6250 --steps 5 --warmup 1 > $out/b1_nodeep.log 2>&1 || exit 1
echo "baseline (no deep-ring tiles in the tuner, epi 24): $(grep -o '"value": [0-9.]*' $out/b1_nodeep.log)"
for v in ${VARIANTS:-24 18 14 28}; do
  DDL_SPLITK_EPI=$v timeout -k 10 300 python bench.py --clients 1 --train-size 6250 --steps 5 --warmup 1 > $out/b1_$v.log 2>&1 || { tail -5 $out/b1_$v.log; exit 1; }
  echo "epi=$v 1 client: $(grep -o '"value": [0-9.]*' $out/b1_$v.log)"
  DDL_SPLITK_EPI=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/p$v -o run -- python bench.py --clients 1 --train-size 6250 --steps 2 --warmup 1 > $out/p$v.log 2>&1 || { tail -5 $out/p$v.log; exit 1; }
  f=$(find $out/p$v -name '*kernel_stats.csv' | head -1)
  python scripts/prof_summary.py "$f" 12 > $out/p${v}_summary.txt
  grep -i "epilogue\|total" $out/p${v}_summary.txt
  find $out/p$v -name '*kernel_trace.csv' -delete
done
echo DONE
