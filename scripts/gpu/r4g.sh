#!/bin/bash
# in-kernel WGRAD split-K fold: numerics (fp32 suites), headline + 1-client bench, A/B with the
# reduce pass (DDL_F32_WG_FOLD=0), GAN fixes
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=r4g
step() {  # name timeout cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > gpurun_out/${T}_${name}.log 2>&1
  local rc=$?
  echo "[$name] rc=$rc :: $(grep -E '^\{|passed|failed' gpurun_out/${T}_${name}.log | tail -2 | cut -c1-330)"
  case $rc in 124|134|137|139) echo "[$name] crashed or timed out: stopping"; exit $rc;; esac
  return 0
}
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
step tests 600 $PT tests/test_fp32_gpu.py tests/test_x6h_gpu.py tests/test_multirank_gpu.py -k "not gan and not vfl"
step gantest 300 $PT tests/test_dcgan.py tests/test_graphs_gpu.py -k "gan"
step bench 300 python -u bench.py --steps 5 --warmup 2
step bench_c1 300 python -u bench.py --clients 1 --train-size 6250 --steps 5 --warmup 2
export DDL_F32_WG_FOLD=0
step bench_nofold 300 python -u bench.py --steps 5 --warmup 2
step bench_c1_nofold 300 python -u bench.py --clients 1 --train-size 6250 --steps 5 --warmup 2
unset DDL_F32_WG_FOLD
step gan 300 python -u benchmarks/bench_vfl_gan.py
