"""BASELINE config #3: data-parallel all-reduce SGD, ResNet-50 ImageNet-shape, one rank per GPU.

Each rank: native ResNet-50 (MFMA implicit-GEMM convs, fused BN; fp32 activations and weights by
default — the reference's precision — or --precision bf16: bf16 activations, fp32 master weights)
on its own synthetic 224x224x3 batch; gradients all-reduced over RCCL in layer-aligned
buckets launched from the backward pass (overlapped); SGD momentum 0.9, wd 1e-4. Weak scaling
(fixed per-GPU batch). value = images/s over all GPUs.

    python benchmarks/bench_resnet50_dp.py --batch 256 --steps 10 --warmup 3
    python -m torch.distributed.run --nproc-per-node 8 benchmarks/bench_resnet50_dp.py ...
"""
from __future__ import annotations

import argparse

import numpy as np
import torch

from _common import emit, timed


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256, help="per-GPU batch")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--pool", type=int, default=1024, help="distinct synthetic images per rank")
    ap.add_argument("--bucket-mb", type=float, default=25.0,
                    help="bucket ceiling: layer-aligned buckets close at 0.64x (16-25 MB by default)")
    ap.add_argument("--precision", default="fp32", choices=("fp32", "bf16"))
    args = ap.parse_args()
    from ddl25spring_amd.data.images import DeviceImageDataset, ImageArrays
    from ddl25spring_amd.models import resnet50_imagenet
    from ddl25spring_amd.optim import SGD
    from ddl25spring_amd.parallel.dp import NativeGradBucketer
    from ddl25spring_amd.runtime import dist as rdist
    ctx = rdist.init()
    dev = ctx.device
    rng = np.random.default_rng(ctx.rank)
    arr = ImageArrays(rng.integers(0, 256, (args.pool, 224, 224, 3), dtype=np.uint8),
                      rng.integers(0, 1000, args.pool), "imagenet", True)
    net = resnet50_imagenet(groups=1, precision=args.precision).to(dev, seed=0)
    ctx.broadcast(net.store.data, 0)
    ctx.broadcast(net.store.buffers, 0)
    net.store.sync_shadow()
    data = DeviceImageDataset(arr, dev, net.input_spec)
    opt = SGD(net, lr=0.1, momentum=0.9, weight_decay=1e-4)
    bk = NativeGradBucketer(net, ctx, bucket_mb=args.bucket_mb)
    net.grad_hook = bk.on_layer_done
    g = torch.Generator(device=dev).manual_seed(1234 + ctx.rank)

    def step():
        idx = torch.randint(0, args.pool, (1, args.batch), device=dev, generator=g, dtype=torch.int32)
        x, y = data.batch(idx)
        opt.zero_grad()
        net.train_step(x, y)
        bk.finish()
        opt.step()

    dt = timed(ctx, step, args.steps, args.warmup)
    ips = ctx.world * args.batch * args.steps / dt
    # all-reduce bus bandwidth on the gradient buffer itself (25.6M fp32), as the rccl-tests
    # convention: busbw = bytes / t * 2 (W - 1) / W; no communication at W = 1
    busbw = None
    if ctx.world > 1:
        g = net.store.grad
        t_ar = timed(ctx, lambda: ctx.all_reduce(g), 10, 3)
        busbw = g.numel() * 4 * 10 / t_ar * 2 * (ctx.world - 1) / ctx.world / 1e9
    emit(ctx, metric="ResNet-50 DP all-reduce SGD images/s (ImageNet-shape)", value=round(ips, 1),
         unit="images/s", n_gpus=ctx.world, steps=args.steps, warmup=args.warmup,
         ms_per_step=round(1e3 * dt / args.steps, 3), higher_is_better=True, scaling="weak",
         vs_baseline=None, dtype=args.precision, data="synthetic",
         allreduce_busbw_GBps=None if busbw is None else round(busbw, 1),
         buckets_mb=[round((hi - lo) * 4 / 2 ** 20, 2) for lo, hi in bk.bounds],
         config={"model": "resnet50-imagenet", "global_batch": ctx.world * args.batch,
                 "seq_len": None, "parallelism": f"dp{ctx.world}", "per_gpu_batch": args.batch})
    rdist.shutdown()


if __name__ == "__main__":
    main()
