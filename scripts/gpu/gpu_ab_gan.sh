#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 200 python benchmarks/bench_vfl_gan.py > gpurun_out/gan_new$i.log 2>&1 && grep -o '"gan_images_per_s": [0-9.]*' gpurun_out/gan_new$i.log || exit 1
(cd scratch/oldtree && timeout -k 10 200 python benchmarks/bench_vfl_gan.py > ../../gpurun_out/gan_old$i.log 2>&1) && grep -o '"gan_images_per_s": [0-9.]*' gpurun_out/gan_old$i.log || exit 1
done
