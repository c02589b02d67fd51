"""BASELINE config #5: vertical-FL split-NN (2-party feature split) + federated DCGAN.

split-NN: heart-disease table (real CSV if present, else synthetic of the same schema), 2 parties
with the D6 balanced feature split, batch 64, AdamW. world 2: rank 0 = active party (labels +
feature block 0), rank 1 = passive party (block 1), cut-layer tensors over RCCL P2P; world 1: both
parties in one process. Metric: samples/s of split-NN training.
DCGAN: CIFAR-10-shaped 32x32x3, 2 clients (one per rank at world 2), FedAvg of G and D every
``--local-steps`` Adam steps. Metric: GAN images/s (real + fake images through D per step), fp32
(the reference's precision, on the main line) and bf16 (a second, labelled line).
"""
from __future__ import annotations

import argparse

import numpy as np
import torch

from _common import emit, timed


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3, help="timed units (split-NN epochs / GAN rounds)")
    ap.add_argument("--warmup", type=int, default=2,
                    help="untimed units (the first runs eagerly, the second captures the HIP graphs)")
    ap.add_argument("--local-steps", type=int, default=20)
    ap.add_argument("--gan-batch", type=int, default=128)
    ap.add_argument("--vfl-batch", type=int, default=64)
    ap.add_argument("--vfl-engine", choices=("fused", "graph"), default="fused",
                    help="world 1: one-launch epoch kernel, or the module path replayed from a HIP graph")
    ap.add_argument("--gan-precisions", default="fp32,bf16",
                    help="DCGAN precisions, the first is the headline line (fp32 = the reference's)")
    args = ap.parse_args()
    from ddl25spring_amd.apps.gan import GANConfig, client_images
    from ddl25spring_amd.data import heart as H
    from ddl25spring_amd.fl.gan import FederatedGAN
    from ddl25spring_amd.models import tabular as T
    from ddl25spring_amd.optim import FlatAdamW
    from ddl25spring_amd.runtime import dist as rdist
    from ddl25spring_amd.runtime.graphs import CapturedStep
    from ddl25spring_amd.vfl import SplitNNParty, SplitNNServer
    ctx = rdist.init()
    dev = ctx.device
    # ---------------- split-NN
    df, real = H.load_heart()
    X, Y = H.vfl_frame(df)
    parts = H.partition_balanced(list(X.columns), 2)
    Xtr, _ = H.row_split(X)
    Ytr, _ = H.row_split(Y)
    xs = [torch.tensor(Xtr[p].values.astype(np.float32), device=dev).contiguous() for p in parts]
    y = torch.tensor(Ytr.values.astype(np.float32), device=dev)
    torch.manual_seed(0)
    bottoms = [T.BottomModel(len(p), 2 * len(p)).to(dev) for p in parts]
    top = T.TopModel(bottoms, 2).to(dev)
    if ctx.world == 1:
        net = T.VFLNetwork(bottoms, 2).to(dev)
        net.top_model = top
        # the framework's fused AdamW (one launch per step, device-side step counter) and fused
        # soft-target CE; on the GPU an epoch (13 fixed-order mini-batches, vfl.py:58-82)
        # replays from one HIP graph
        net.optimizer = FlatAdamW(net.parameters()) if dev.type == "cuda" else torch.optim.AdamW(net.parameters())
        crit = T.SoftCrossEntropy()

        def one_epoch():
            for b in range(0, len(y), args.vfl_batch):
                net.optimizer.zero_grad()
                crit(net([x[b:b + args.vfl_batch] for x in xs]), y[b:b + args.vfl_batch]).backward()
                net.optimizer.step()

        eng = net.fused_epoch_engine(args.vfl_batch) if args.vfl_engine == "fused" else None
        if eng is not None:
            # the whole epoch (13 mini-batches: forward, CE, backward, AdamW) in one launch,
            # csrc/kernels/mlp_epoch.hip
            stats = torch.zeros(2, device=dev)

            def epoch():
                eng.run(xs, y, stats)
        else:
            epoch = CapturedStep(one_epoch, warmup=1, enabled=dev.type == "cuda")
    elif ctx.rank == 0:
        srv = SplitNNServer(top, [1], [2 * len(parts[1])], local_bottom=bottoms[0])

        def epoch():
            srv.fit(y, 1, args.vfl_batch, x_local=xs[0])
    else:
        pty = SplitNNParty(bottoms[1], 2 * len(parts[1]))

        def epoch():
            pty.fit(xs[1], 1, args.vfl_batch)
    dt_v = timed(ctx, epoch, args.steps, args.warmup)
    vfl_sps = len(y) * args.steps / dt_v
    # ---------------- federated DCGAN (2 clients): fp32 (the reference's precision) first, then bf16
    gcfg = GANConfig(clients=2, local_steps=args.local_steps, batch_size=args.gan_batch,
                     train_size=10000)
    data = client_images(gcfg, dev)
    gan = {}
    for prec in args.gan_precisions.split(","):
        fg = FederatedGAN(data, ctx=ctx, local_steps=args.local_steps,
                          batch_size=args.gan_batch, device=dev, precision=prec)
        fg.run(args.warmup)
        # timed rounds enqueue without host syncs (device-made inputs, native aggregation); the
        # losses are read once when run() returns
        fg.sync_rounds = False
        dt = timed(ctx, lambda: fg.run(args.steps), 1, 0)
        gan[prec] = dt
    imgs = 2 * 2 * args.local_steps * args.gan_batch * args.steps  # 2 clients x (real + fake)
    precs = list(gan)
    emit(ctx, metric="VFL split-NN samples/s + federated DCGAN images/s", value=round(vfl_sps, 1),
         unit="samples/s", n_gpus=ctx.world, steps=args.steps, warmup=args.warmup,
         ms_per_step=round(1e3 * dt_v / args.steps, 3), higher_is_better=True, scaling="strong",
         vs_baseline=None, dtype=f"fp32 (split-NN) / {precs[0]} (DCGAN)",
         data="heart.csv" if real else "synthetic",
         vfl_engine="fused-epoch-kernel" if ctx.world == 1 and args.vfl_engine == "fused" and dev.type == "cuda"
         else ("hip-graph" if ctx.world == 1 else "rccl-p2p"),
         gan_images_per_s=round(imgs / gan[precs[0]], 1), gan_ms_per_round=round(1e3 * gan[precs[0]] / args.steps, 3),
         config={"model": "splitnn-heart-2party + dcgan-cifar32", "global_batch": args.vfl_batch,
                 "seq_len": None, "parallelism": f"vfl2party-fedgan2-w{ctx.world}"})
    for prec in precs[1:]:  # labelled extra lines (the faster non-reference precision)
        emit(ctx, metric="federated DCGAN images/s", value=round(imgs / gan[prec], 1), unit="images/s",
             n_gpus=ctx.world, steps=args.steps, warmup=args.warmup,
             ms_per_step=round(1e3 * gan[prec] / args.steps, 3), higher_is_better=True, scaling="strong",
             vs_baseline=None, dtype=prec, data="synthetic",
             config={"model": "dcgan-cifar32", "global_batch": 2 * args.gan_batch, "seq_len": None,
                     "parallelism": f"fedgan2-w{ctx.world}"})
    rdist.shutdown()


if __name__ == "__main__":
    main()
