set -o pipefail
bash scripts/gpu/gpu_ab_f32.sh "cur w128" "fwd" "c64 c256 c512" w128 > gpurun_out/w128_ab.txt 2>&1 || exit 1
bash scripts/gpu/pmc_f32_mem.sh abvar/w128.so fwd c64 > gpurun_out/pmcm_fwd64_w128.txt 2>&1
