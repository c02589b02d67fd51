#!/bin/bash
# IPC peer-read all-reduce tests (ranks share the one GPU) + round-graph FL tests and benches.
set -o pipefail
tag=${1:-ipc}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -h '^{' "$out/$name.log" | cut -c1-150; tail -n 3 "$out/$name.log" | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
step ipc 300 python -u -m pytest tests/test_ipc_gpu.py -x -v --timeout 200 --timeout-method thread
