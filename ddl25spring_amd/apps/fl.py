"""Horizontal FL experiment runner (reference hfl_complete.py __main__ / homework-1 sweeps).

One process per GPU (or CPU/gloo ranks); the FL round protocol, client sampling and RunResult
table are the reference's; the model, aggregator, attack and failures are configurable.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np


@dataclass
class FLConfig:
    algorithm: str = "fedavg"      # fedavg | fedsgd | fedsgd_weight
    model: str = "mnist_cnn"       # mnist_cnn | mnist_mlp | resnet18 | resnet50
    dataset: str = "mnist"         # mnist | cifar10 | imagenet (real copy via DDL_DATA_ROOT, else synthetic)
    clients: int = 100
    client_fraction: float = 0.1
    batch_size: int = 100          # -1 = infinity (full local batch)
    local_epochs: int = 1
    lr: float = 0.01
    rounds: int = 10
    iid: bool = True
    seed: int = 10
    aggregator: str = "mean"       # mean | median | trimmed_mean | krum | multi_krum
    trim: float = 0.1
    krum_f: int = 1
    attack: str | None = None      # label_flip | sign_flip | gaussian | free_rider
    malicious: int = 0             # number of malicious clients (ids 0..malicious-1)
    dropout: float = 0.0
    stragglers: float = 0.0        # probability a sampled client is slow
    straggler_slowdown: float = 4.0
    deadline: float | None = None  # drop clients slower than this (x nominal mean-shard time)
    train_size: int | None = None
    test_size: int | None = None
    checkpoint: str | None = None
    jsonl: str | None = None


def build_server(cfg: FLConfig, ctx):
    from ..data.images import DeviceImageDataset, load_images
    from ..data.split import split
    from ..fl.algorithms import FedAvg, FedSGD, FedSgdWeight
    from ..fl.attacks import make_attack
    from ..models import mnist_cnn, mnist_mlp, resnet18_cifar, resnet50_imagenet
    train = load_images(cfg.dataset, True, cfg.train_size, seed=cfg.seed)
    test = load_images(cfg.dataset, False, cfg.test_size, seed=cfg.seed)
    parts = split(cfg.clients, cfg.iid, cfg.seed, labels=train.labels)
    model_fn = {"mnist_cnn": mnist_cnn, "mnist_mlp": mnist_mlp, "resnet18": resnet18_cifar,
                "resnet50": resnet50_imagenet}[cfg.model]
    attack = make_attack(cfg.attack, list(range(cfg.malicious))) if cfg.attack else None
    algo = {"fedavg": FedAvg, "fedsgd": FedSGD, "fedsgd_weight": FedSgdWeight}[cfg.algorithm]
    kw = dict(lr=cfg.lr, client_fraction=cfg.client_fraction, seed=cfg.seed,
              test_data=DeviceImageDataset(test, ctx.device), aggregator=cfg.aggregator,
              agg_kwargs={"trim": cfg.trim, "f": cfg.krum_f}, attack=attack, ctx=ctx,
              dropout=cfg.dropout, stragglers=cfg.stragglers,
              straggler_slowdown=cfg.straggler_slowdown, deadline=cfg.deadline)
    if algo is FedAvg:
        kw.update(batch_size=cfg.batch_size, local_epochs=cfg.local_epochs)
    return algo(model_fn, DeviceImageDataset(train, ctx.device), parts, **kw)


def run_fl(cfg: FLConfig, ctx, log=print):
    from ..fl import checkpoint as ckpt
    from ..utils.metrics import JsonlLogger
    server = build_server(cfg, ctx)
    if cfg.checkpoint:
        res = ckpt.run_with_checkpoints(server, cfg.rounds, cfg.checkpoint)
    else:
        res = server.run(cfg.rounds)
    with JsonlLogger(cfg.jsonl, ctx.rank) as jl:
        for i in range(len(res.test_accuracy)):
            rec = dict(round=i + 1, test_accuracy=res.test_accuracy[i],
                       message_count=res.message_count[i])
            if i < len(res.round_time):
                rec.update(round_time=res.round_time[i], samples=res.samples[i],
                           samples_per_s=res.samples[i] / max(res.round_time[i], 1e-9))
            if i < len(res.phase_ms):
                rec["phase_ms"] = res.phase_ms[i]
            jl.log(**rec)
    if log and ctx.rank == 0:
        log(res.as_df(with_throughput=True).to_string(index=False))
        if np.isfinite(res.test_accuracy[-1]):
            log(f"final test accuracy {res.test_accuracy[-1]:.2f}%")
    return res
