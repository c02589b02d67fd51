"""Federated DCGAN program (BASELINE config "federated DCGAN"): CIFAR-10-shaped images (real copy
via DDL_DATA_ROOT, else synthetic), IID shards, FedAvg over G and D every ``local_steps``."""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch


@dataclass
class GANConfig:
    clients: int = 2
    client_fraction: float = 1.0
    rounds: int = 10
    local_steps: int = 50
    batch_size: int = 64
    lr: float = 2e-4
    ngf: int = 64
    ndf: int = 64
    train_size: int = 50000
    seed: int = 0
    save: str = ""  # rank 0 writes the final flat global (G | D | BN) weights here (torch.save)
    ckpt_dir: str = ""  # per-rank sharded checkpoint (runtime/checkpoint.py); resumes if committed
    ckpt_every: int = 0  # commit every N rounds (0: only at the end)
    precision: str = "fp32"  # fp32 (the reference's generative lab) | bf16


def client_images(cfg: GANConfig, device):
    from ..data.images import load_images
    from ..data.split import split
    from ..models.dcgan import to_nhwc_padded
    arr = load_images("cifar10", True, cfg.train_size, seed=cfg.seed)
    imgs = torch.from_numpy(np.ascontiguousarray(arr.images)).float().div_(127.5).sub_(1.0)  # NHWC
    parts = split(cfg.clients, True, cfg.seed, labels=arr.labels)
    return [to_nhwc_padded(imgs[torch.from_numpy(p)].permute(0, 3, 1, 2)).to(device) for p in parts]


def run_gan(cfg: GANConfig, ctx, log=print):
    from ..fl.gan import FederatedGAN
    data = client_images(cfg, ctx.device)
    fg = FederatedGAN(data, ctx=ctx, ngf=cfg.ngf, ndf=cfg.ndf, lr=cfg.lr,
                      local_steps=cfg.local_steps, batch_size=cfg.batch_size,
                      client_fraction=cfg.client_fraction, seed=cfg.seed, device=ctx.device,
                      precision=cfg.precision)
    ckpt = None
    if cfg.ckpt_dir:
        from ..runtime.checkpoint import ShardedCheckpoint
        tag = (f"gan,clients={cfg.clients},C={cfg.client_fraction},bs={cfg.batch_size},ls={cfg.local_steps},"
               f"seed={cfg.seed},prec={cfg.precision}")
        ckpt = ShardedCheckpoint(cfg.ckpt_dir, ctx, tag=tag)
        got = ckpt.load()
        if got is not None:
            fg.load_state_dict(got[1])
    from ..fl.gan import GANRunResult
    res = GANRunResult()
    while fg.round_idx < cfg.rounds:
        part = fg.run(1)
        res.rounds += part.rounds
        res.loss_d += part.loss_d
        res.loss_g += part.loss_g
        res.wall_time += part.wall_time
        res.samples += part.samples
        if ckpt is not None and ((cfg.ckpt_every and fg.round_idx % cfg.ckpt_every == 0)
                                 or fg.round_idx == cfg.rounds):
            ckpt.save(fg.round_idx, fg.state_dict())
    if log and ctx.rank == 0:
        for r, (ld, lg, t) in enumerate(zip(res.loss_d, res.loss_g, res.wall_time)):
            log(f"round {r + 1}: loss_D {ld:.3f} loss_G {lg:.3f} ({t:.2f}s)")
    if cfg.save and ctx.rank == 0:
        torch.save(fg._flat().detach().cpu(), cfg.save)
    return res
