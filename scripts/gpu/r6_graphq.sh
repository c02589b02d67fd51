#!/bin/bash
# HIP-graph execution knobs A/B on the 1-client and 8-client FedAvg steps
set -o pipefail
mkdir -p gpurun_out
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py $ARGS > gpurun_out/gq_${tag}.log 2>&1 || { tail -5 gpurun_out/gq_${tag}.log; return 1; }
  echo "$tag $(grep '^{' gpurun_out/gq_${tag}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
ARGS="--clients 1 --train-size 6250 --steps 5 --warmup 1"
run c1_base A=1 && run c1_q1 DEBUG_HIP_FORCE_GRAPH_QUEUES=1 && run c1_q2 DEBUG_HIP_FORCE_GRAPH_QUEUES=2 && \
run c1_pc1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 && run c1_pc0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 && \
run c1_q1_noov DEBUG_HIP_FORCE_GRAPH_QUEUES=1 DDL_WGRAD_OVERLAP=0 && run c1_base2 A=1
