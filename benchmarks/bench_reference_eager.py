"""Reference-equivalent FedAvg loop in stock PyTorch-ROCm: the throughput baseline of BASELINE.md.

The reference publishes no throughput (BASELINE.json ``published = {}``), so the number our
``bench.py`` is compared against is the reference's own FedAvg loop run on the same MI355X with the
same config (ResNet-18, CIFAR-10 shape, 8 IID clients, B=100, E=1, lr=0.01, 50k samples/round):

  * ``faithful`` — ``FedAvgServer.run`` as written (lab/tutorial_1a/hfl_complete.py:347-390):
    server weights snapshot to the host (:356); clients run one after another (:360-373), each an
    ``nn.Module`` replica fed by a shuffling DataLoader (:146-151) that copies every batch to the
    device, ``train_epoch`` with ``zero_grad / forward / loss / backward / SGD.step`` (:71-80);
    weights copied back to the host (:332); ``n_k``-weighted sum on the host (:370-378) and the
    average copied back to the device (:380-383). fp32, NCHW, MIOpen convs.
  * ``tuned`` — the same algorithm with the usual eager-PyTorch speedups and no host round trips:
    data resident on the device, bf16 autocast, channels_last, aggregation on the device;
  * ``tuned_fp32`` — as ``tuned`` at the reference's precision (no autocast; MIOpen fp32 convs with
    cudnn.benchmark): the strongest stock-PyTorch fp32 loop, the fair comparison for bench.py's
    fp32 headline.

Both use synthetic CIFAR-shaped tensors (pre-normalised) and random init (no network here).

    python benchmarks/bench_reference_eager.py --variant faithful --steps 1 --warmup 1
"""
from __future__ import annotations

import argparse
import time

import numpy as np
import torch
import torch.nn.functional as F
from _common import emit

from ddl25spring_amd.models.torch_ref import torch_resnet18_cifar

METRIC = "FedAvg rounds/sec + local samples/sec, ResNet-18 CIFAR-10-shape, 8 clients"


def make_data(n, device, seed=0):
    g = torch.Generator().manual_seed(seed)
    y = torch.randint(0, 10, (n,), generator=g)
    x = torch.randn(n, 3, 32, 32, generator=g) * 0.5
    x += 0.25 * (y.float()[:, None, None, None] / 9.0 - 0.5)  # weakly learnable
    return x.to(device), y.to(device)


class Client:
    """WeightClient (hfl_complete.py:316-332): own model replica + own shuffling loader."""

    def __init__(self, x, y, idx, lr, B, E, device, tuned, amp=True):
        self.x, self.y, self.idx = x, y, idx
        self.B, self.E, self.device, self.tuned, self.amp = B, E, device, tuned, amp
        self.model = torch_resnet18_cifar().to(device)
        if tuned:
            self.model = self.model.to(memory_format=torch.channels_last)
        self.opt = torch.optim.SGD(self.model.parameters(), lr=lr)
        self.gen = torch.Generator()

    def update(self, weights, seed):
        with torch.no_grad():
            for p, w in zip(self.model.state_dict().values(), weights):
                p.copy_(w)  # host -> device in the faithful variant
        self.gen.manual_seed(seed)
        self.model.train()
        n = 0
        for _ in range(self.E):
            perm = self.idx[torch.randperm(len(self.idx), generator=self.gen)]
            for s in range(0, len(perm), self.B):
                bi = perm[s:s + self.B]
                if self.tuned:
                    xb, yb = self.x[bi.to(self.x.device)], self.y[bi.to(self.y.device)]
                else:  # DataLoader: host batch -> device
                    xb, yb = self.x[bi].to(self.device), self.y[bi].to(self.device)
                self.opt.zero_grad()
                if self.tuned:
                    xb = xb.contiguous(memory_format=torch.channels_last)
                    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=self.amp):
                        loss = F.cross_entropy(self.model(xb), yb)
                else:
                    loss = F.cross_entropy(self.model(xb), yb)
                loss.backward()
                self.opt.step()
                n += len(bi)
        sd = self.model.state_dict().values()
        if self.tuned:
            return [t.detach().clone() for t in sd], n
        return [t.detach().cpu().clone() for t in sd], n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", choices=("faithful", "tuned", "tuned_fp32"), default="faithful")
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--clients", type=int, default=8)
    ap.add_argument("--batch", type=int, default=100)
    ap.add_argument("--epochs", type=int, default=1)
    ap.add_argument("--lr", type=float, default=0.01)
    ap.add_argument("--train-size", type=int, default=50000)
    args = ap.parse_args()
    from ddl25spring_amd.runtime import dist as rdist
    ctx = rdist.init()
    dev = ctx.device
    tuned = args.variant in ("tuned", "tuned_fp32") and dev.type == "cuda"
    amp = args.variant == "tuned"
    torch.backends.cudnn.benchmark = tuned
    torch.backends.cudnn.deterministic = not tuned  # hfl_complete.py:17
    x, y = make_data(args.train_size, dev if tuned else "cpu")
    perm = torch.from_numpy(np.random.default_rng(10).permutation(args.train_size))
    shards = torch.tensor_split(perm, args.clients)
    # this rank's clients (one GPU = one group of client slots, as in bench.py)
    mine = [c for c in range(args.clients) if c % ctx.world == ctx.rank]
    torch.manual_seed(10)
    server = torch_resnet18_cifar().to(dev)
    clients = {c: Client(x, y, shards[c], args.lr, args.batch, args.epochs, dev, tuned, amp) for c in mine}
    sizes = torch.tensor([len(s) for s in shards], dtype=torch.float64)
    p = (sizes / sizes.sum()).tolist()

    def one_round(r):
        sd = server.state_dict()
        weights = [t.detach().clone() if tuned else t.detach().cpu().clone() for t in sd.values()]
        acc, samples = None, 0
        for c in mine:
            w, n = clients[c].update(weights, 10 + c + 1 + r * args.clients)
            samples += n
            scaled = [t * p[c] if t.is_floating_point() else t for t in w]
            acc = scaled if acc is None else [a + b if a.is_floating_point() else b
                                              for a, b in zip(acc, scaled)]
        if ctx.world > 1:  # the server's weighted reduce across the GPUs holding the clients
            for t in acc:
                if t.is_floating_point():
                    tt = t.to(dev)
                    torch.distributed.all_reduce(tt)
                    t.copy_(tt)
        with torch.no_grad():
            for t, a in zip(sd.values(), acc):
                t.copy_(a)  # host -> device in the faithful variant
        return samples

    for r in range(args.warmup):
        one_round(r)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    ctx.barrier()
    t0 = time.perf_counter()
    samples = 0
    for r in range(args.steps):
        samples += one_round(args.warmup + r)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    ctx.barrier()
    dt = ctx.max_scalar(time.perf_counter() - t0)
    samples = int(ctx.sum_scalar(samples))
    emit(ctx, metric=METRIC + f" [reference-equivalent eager PyTorch, {args.variant}]",
         value=round(samples / dt, 1), unit="samples/s", n_gpus=ctx.world, steps=args.steps,
         warmup=args.warmup, ms_per_step=round(1e3 * dt / args.steps, 3), higher_is_better=True,
         scaling="strong", vs_baseline=None, dtype="bf16-autocast" if (tuned and amp) else "fp32",
         data="synthetic", rounds_per_sec=round(args.steps / dt, 4),
         config={"model": "resnet18-cifar10", "global_batch": args.batch * args.clients,
                 "seq_len": None, "parallelism": f"fedavg-{args.clients}clients-eager-w{ctx.world}",
                 "variant": args.variant})
    rdist.shutdown()


if __name__ == "__main__":
    main()
