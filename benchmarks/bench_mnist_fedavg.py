"""FedAvg on the reference's own workload: MnistCnn on MNIST-shaped data with homework-1's default
configuration (lab/homework-1.ipynb:50-59: N=100 clients, C=0.1 -> K=10 sampled per round, E=1,
B=100, lr=0.01, seed 10; 600 samples per client).

  * ``native``   — this framework: ``fl.algorithms.FedAvg`` on the client-batched engine (the 10
                   sampled clients train as one group of slots, weights resident in HBM, the
                   round's local steps replayed as one HIP graph, device-side weighted reduce).
  * ``faithful`` — the reference loop as written (hfl_complete.py:336-390) in stock PyTorch-ROCm:
                   server weights to the host, the sampled clients one after another, each an
                   ``nn.Module`` replica fed by a shuffling loader that copies every batch to the
                   device, weights back to the host, the n_k-weighted sum on the host. fp32.

Synthetic MNIST-shaped uint8 images (learnable class templates), random init.

    python benchmarks/bench_mnist_fedavg.py --variant native --steps 10 --warmup 2 [--precision bf16]

The native variant defaults to fp32 (the reference's precision); ``--precision bf16`` is the
labelled faster mode.
"""
from __future__ import annotations

import argparse
import time

import numpy as np
import torch
import torch.nn.functional as F
from _common import emit

METRIC = "FedAvg rounds/sec + local samples/sec, MnistCnn MNIST-shape, N=100 C=0.1 (homework-1 defaults)"


def run_native(args, ctx):
    from ddl25spring_amd.data.images import DeviceImageDataset, synthetic_images
    from ddl25spring_amd.data.split import split
    from ddl25spring_amd.fl.algorithms import FedAvg
    from ddl25spring_amd.models import mnist_cnn
    train = synthetic_images("mnist", args.train_size, seed=0)
    parts = split(args.clients, True, 10, labels=train.labels)
    def model(groups=1):
        return mnist_cnn(groups, precision=args.precision)
    fl = FedAvg(model, DeviceImageDataset(train, ctx.device), parts, lr=args.lr,
                batch_size=args.batch, local_epochs=args.epochs, client_fraction=args.fraction,
                seed=10, eval_every=0)
    for _ in range(args.warmup):
        fl.round()
    if ctx.device.type == "cuda":
        torch.cuda.synchronize()
    ctx.barrier()
    t0 = time.perf_counter()
    samples = 0
    for _ in range(args.steps):
        samples += fl.round()[1]
    if ctx.device.type == "cuda":
        torch.cuda.synchronize()
    ctx.barrier()
    return ctx.max_scalar(time.perf_counter() - t0), samples


def run_faithful(args, ctx):
    from ddl25spring_amd.data.images import SHAPES, synthetic_images
    from ddl25spring_amd.data.split import split
    from ddl25spring_amd.models.torch_ref import TorchMnistCnn
    dev = ctx.device
    torch.backends.cudnn.deterministic = True  # hfl_complete.py:17
    train = synthetic_images("mnist", args.train_size, seed=0)
    mean, std = SHAPES["mnist"][6][0], SHAPES["mnist"][7][0]
    x_host = (torch.from_numpy(train.images).float().permute(0, 3, 1, 2) / 255.0 - mean) / std
    y_host = torch.from_numpy(train.labels)
    parts = [torch.as_tensor(p) for p in split(args.clients, True, 10, labels=train.labels)]
    rng = np.random.default_rng(10)
    K = max(1, round(args.fraction * args.clients))
    torch.manual_seed(10)
    server = TorchMnistCnn().to(dev)
    models: dict = {}

    def client_update(c, weights, seed):  # WeightClient.update (hfl_complete.py:322-332)
        if c not in models:
            m = TorchMnistCnn().to(dev)
            models[c] = (m, torch.optim.SGD(m.parameters(), lr=args.lr))
        m, opt = models[c]
        with torch.no_grad():
            for p, w in zip(m.parameters(), weights):
                p.copy_(w)  # host -> device
        g = torch.Generator().manual_seed(seed)
        m.train()
        idx = parts[c]
        for _ in range(args.epochs):  # train_epoch over a DataLoader(shuffle=True, generator=g)
            perm = idx[torch.randperm(len(idx), generator=g)]
            for s in range(0, len(perm), args.batch):
                bi = perm[s:s + args.batch]
                xb, yb = x_host[bi].to(dev), y_host[bi].to(dev)
                opt.zero_grad()
                F.nll_loss(m(xb), yb).backward()
                opt.step()
        return [p.detach().cpu().clone() for p in m.parameters()], len(idx) * args.epochs

    def one_round(r):
        weights = [p.detach().cpu().clone() for p in server.parameters()]  # :356
        chosen = rng.choice(args.clients, K, replace=False)
        tot = float(sum(len(parts[c]) for c in chosen))
        acc, samples = None, 0
        for i, c in enumerate(chosen):
            w, n = client_update(int(c), weights, 10 + int(c) + 1 + r * K)
            samples += n
            scaled = [t * (len(parts[c]) / tot) for t in w]
            acc = scaled if acc is None else [a + b for a, b in zip(acc, scaled)]
        with torch.no_grad():
            for p, a in zip(server.parameters(), acc):
                p.copy_(a.to(dev))  # :380-383
        return samples

    for r in range(args.warmup):
        one_round(r)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    samples = sum(one_round(args.warmup + r) for r in range(args.steps))
    if dev.type == "cuda":
        torch.cuda.synchronize()
    return time.perf_counter() - t0, samples


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", choices=("native", "faithful"), default="native")
    ap.add_argument("--steps", type=int, default=10, help="timed FedAvg rounds")
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--clients", type=int, default=100)
    ap.add_argument("--fraction", type=float, default=0.1)
    ap.add_argument("--batch", type=int, default=100)
    ap.add_argument("--epochs", type=int, default=1)
    ap.add_argument("--lr", type=float, default=0.01)
    ap.add_argument("--train-size", type=int, default=60000)
    ap.add_argument("--precision", choices=("fp32", "bf16"), default="fp32",
                    help="native variant: fp32 = the reference's precision (default), bf16 = bf16 MFMA")
    args = ap.parse_args()
    from ddl25spring_amd.runtime import dist as rdist
    ctx = rdist.init()
    if args.variant == "faithful" and ctx.world > 1:
        raise SystemExit("the faithful reference loop is single-process")
    dt, samples = (run_native if args.variant == "native" else run_faithful)(args, ctx)
    emit(ctx, metric=METRIC, variant=args.variant, value=round(samples / dt, 1), unit="samples/s",
         rounds_per_sec=round(args.steps / dt, 3), n_gpus=ctx.world, steps=args.steps,
         warmup=args.warmup, ms_per_step=round(1e3 * dt / args.steps, 3), higher_is_better=True,
         dtype=args.precision if args.variant == "native" else "fp32", data="synthetic",
         config={"model": "mnist_cnn", "clients": args.clients, "client_fraction": args.fraction,
                 "local_batch": args.batch, "local_epochs": args.epochs, "lr": args.lr})
    rdist.shutdown()


if __name__ == "__main__":
    main()
