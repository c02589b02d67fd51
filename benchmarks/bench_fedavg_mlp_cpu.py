"""BASELINE config #1: FedAvg 2-client MLP on MNIST-shaped tensors, CPU / gloo (tutorial_1a
plumbing, no GPU). Run with 2 ranks (one client each) through the launcher or torchrun, or 1 rank
(both clients client-batched in one process)."""
from __future__ import annotations

import argparse

from _common import emit


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--train-size", type=int, default=60000)
    args = ap.parse_args()
    from ddl25spring_amd.data.images import DeviceImageDataset, load_images
    from ddl25spring_amd.data.split import split
    from ddl25spring_amd.fl.algorithms import FedAvg
    from ddl25spring_amd.models import mnist_mlp
    from ddl25spring_amd.runtime import dist as rdist
    ctx = rdist.init(backend="gloo", device="cpu")
    # torchrun exports OMP_NUM_THREADS=1 to every rank; give each rank its share of the cores
    import os
    import torch
    torch.set_num_threads(max(1, (os.cpu_count() or 1) // ctx.world))
    train = load_images("mnist", True, args.train_size)
    parts = split(2, True, 10, labels=train.labels)
    fa = FedAvg(mnist_mlp, DeviceImageDataset(train, "cpu"), parts, lr=0.01, batch_size=100,
                client_fraction=1.0, seed=10, ctx=ctx, eval_every=0)
    for _ in range(args.warmup):
        fa.round()
    tot_t, tot_s = 0.0, 0
    for _ in range(args.steps):
        dt, s = fa.round()
        tot_t += dt
        tot_s += s
    emit(ctx, metric="FedAvg rounds/sec + local samples/sec, MLP MNIST-shape, 2 clients (CPU/gloo)",
         value=round(tot_s / tot_t, 1), unit="samples/s", n_gpus=0, ranks=ctx.world,
         steps=args.steps, warmup=args.warmup, ms_per_step=round(1e3 * tot_t / args.steps, 3),
         rounds_per_sec=round(args.steps / tot_t, 4), higher_is_better=True, scaling="strong",
         vs_baseline=None, dtype="fp32", data="synthetic",
         config={"model": "mlp-800-200-200-10", "global_batch": 200, "seq_len": None,
                 "parallelism": f"fedavg-2clients-gloo{ctx.world}"})
    rdist.shutdown()


if __name__ == "__main__":
    main()
