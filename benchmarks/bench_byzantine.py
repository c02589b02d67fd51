"""BASELINE config #4: Byzantine-robust FL — Krum / trimmed-mean / coordinate-median under
label-flip + sign-flip attackers, 8 clients (ResNet-18, CIFAR-10 shape, the headline workload).

Per aggregator: FedAvg rounds/s and the device time of the aggregation phase (coordinate-sharded
all-to-all + bitonic selection / fp32-MFMA Gram kernels), optionally test accuracy (--eval).
"""
from __future__ import annotations

import argparse

import numpy as np

from _common import emit


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=2, help="timed rounds per aggregator")
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--model", default="resnet18")
    ap.add_argument("--train-size", type=int, default=50000)
    ap.add_argument("--aggregators", default="mean,median,trimmed_mean,krum")
    ap.add_argument("--eval", action="store_true")
    args = ap.parse_args()
    from ddl25spring_amd.data.images import DeviceImageDataset, load_images
    from ddl25spring_amd.data.split import split
    from ddl25spring_amd.fl.algorithms import FedAvg
    from ddl25spring_amd.fl.attacks import make_attack
    from ddl25spring_amd.models import mnist_cnn, resnet18_cifar
    from ddl25spring_amd.runtime import dist as rdist
    ctx = rdist.init()
    kind = "cifar10" if args.model == "resnet18" else "mnist"
    model_fn = resnet18_cifar if args.model == "resnet18" else mnist_cnn
    train = load_images(kind, True, args.train_size)
    test = load_images(kind, False, 2000)
    parts = split(8, True, 0, labels=train.labels)
    data, tdata = DeviceImageDataset(train, ctx.device), DeviceImageDataset(test, ctx.device)
    results = {}
    for agg in args.aggregators.split(","):
        # clients 0,1 flip labels, clients 2,3 flip (and scale) their update signs: 4 of 8 hostile
        # for the data-poisoning pair, 2 of 8 model-poisoners
        attack = make_attack("sign_flip", [2, 3])
        fa = FedAvg(model_fn, data, parts, lr=0.01, batch_size=100, client_fraction=1.0, seed=0,
                    test_data=tdata, aggregator=agg, agg_kwargs={"trim": 0.25, "f": 2},
                    attack=attack, ctx=ctx, eval_every=0)
        flip = make_attack("label_flip", [0, 1])
        fa.attack = _Both(attack, flip)
        for _ in range(args.warmup):
            fa.round()
        fa.timer.summary()
        times, agg_ms = [], []
        for _ in range(args.steps):
            dt, _ = fa.round()
            times.append(dt)
            agg_ms.append(fa.timer.summary().get("aggregate", float("nan")))
        results[agg] = {"rounds_per_s": round(len(times) / sum(times), 4),
                        "aggregate_ms": round(float(np.mean(agg_ms)), 3)}
        if args.eval:
            results[agg]["test_accuracy"] = fa.test()
    emit(ctx, metric="Byzantine-robust FedAvg rounds/s (8 clients, 2 label-flip + 2 sign-flip)",
         value=results.get("krum", next(iter(results.values())))["rounds_per_s"], unit="rounds/s",
         n_gpus=ctx.world, steps=args.steps, warmup=args.warmup, higher_is_better=True,
         scaling="strong", vs_baseline=None, dtype="bf16", data="synthetic", per_aggregator=results,
         config={"model": f"{args.model}-{kind}", "global_batch": 800, "seq_len": None,
                 "parallelism": f"fedavg-8clients-dp{ctx.world}"})
    rdist.shutdown()


class _Both:
    """label flip (data poisoning) for some clients + sign flip (model poisoning) for others."""

    def __init__(self, model_attack, data_attack):
        self.m, self.d = model_attack, data_attack

    def label_transform_for(self, mine, ncls):
        return self.d.label_transform_for(mine, ncls)

    def skip_training(self, c):
        return False

    def poison_updates(self, rows, w_global, mine):
        self.m.poison_updates(rows, w_global, mine)


if __name__ == "__main__":
    main()
