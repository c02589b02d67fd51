#!/bin/bash
# Functional rehearsal of bench.py's N>1 path on a one-GPU box: 2 and 4 ranks share cuda:0 over
# gloo (RCCL needs one GPU per rank). Checks the rendezvous, per-rank client split, the cross-rank
# FedAvg aggregation and the max-over-ranks timing line; the numbers are not a scaling result.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/multirank
mkdir -p $out
for n in 2 4; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
      --master-addr 127.0.0.1 --master-port $((29500 + n)) \
      bench.py --gpus $n --steps 2 --warmup 1 --backend gloo > $out/n$n.log 2>&1
  rc=$?
  grep '^{' $out/n$n.log | cut -c1-400
  [ $rc -eq 0 ] || { echo "n=$n rc=$rc"; tail -30 $out/n$n.log; exit $rc; }
done
echo ALLDONE
