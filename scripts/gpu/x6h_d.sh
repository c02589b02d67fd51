set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_x6h_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/x6h_tests.log 2>&1 || { tail -40 gpurun_out/x6h_tests.log; exit 1; }
tail -1 gpurun_out/x6h_tests.log
for L in c64 c128 c256; do for O in fwd dgrad; do
  timeout -k 10 60 python scripts/conv_f32_bench.py --math auto --halo 1 --mode $O --layer $L --reps 20 2>&1 | tail -1 || exit 1
done; done
bash scripts/gpu/fp32_bench_prof.sh r4b
