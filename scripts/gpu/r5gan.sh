#!/bin/bash
# fp32 DCGAN: record its conv launches, graph-timed tune of exactly those, merge, A/B the GAN bench
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
DDL_F32_RECORD=$PWD/gpurun_out/gan_geoms.json timeout -k 10 300 python -u benchmarks/bench_vfl_gan.py --gan-precisions fp32 > gpurun_out/r5gan_b0.log 2>&1 || { tail -5 gpurun_out/r5gan_b0.log; exit 1; }
echo "before $(grep -o '"gan_images_per_s": [0-9.]*' gpurun_out/r5gan_b0.log)"
python -c "import json; print(len(json.load(open('gpurun_out/gan_geoms.json'))), 'launches recorded')"
timeout -k 10 600 python -u scripts/conv_f32_tune.py --geoms-file gpurun_out/gan_geoms.json --math auto --skip-halo --budget-s 500 --out gpurun_out/gan_plans.json > gpurun_out/r5gan_tune.log 2>&1 || { tail -5 gpurun_out/r5gan_tune.log; exit 1; }
tail -1 gpurun_out/r5gan_tune.log
python scripts/merge_plans.py gpurun_out/gan_plans.json && cp ddl25spring_amd/ops/f32_plans.json gpurun_out/f32_plans_gan.json
for r in 1 2; do
timeout -k 10 300 python -u benchmarks/bench_vfl_gan.py --gan-precisions fp32 > gpurun_out/r5gan_b.log 2>&1 || { tail -5 gpurun_out/r5gan_b.log; exit 1; }
echo "after $(grep -o '"gan_images_per_s": [0-9.]*' gpurun_out/r5gan_b.log)"
done
