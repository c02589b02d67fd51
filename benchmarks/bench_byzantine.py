"""BASELINE config #4: Byzantine-robust FL — Krum / trimmed-mean / coordinate-median under
label-flip + sign-flip attackers, 8 clients (ResNet-18, CIFAR-10 shape, the headline workload).

Per aggregator: FedAvg rounds/s and the device time of the aggregation phase (coordinate-sharded
all-to-all + bitonic selection / fp32-MFMA Gram kernels) under attack, and the robustness itself:
test accuracy after ``--acc-rounds`` rounds on the learnable synthetic CIFAR set, clean (no
attacker) vs attacked, for every aggregator (``--no-eval`` skips the accuracy runs).
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
    ap.add_argument("--no-eval", dest="eval", action="store_false")
    ap.add_argument("--acc-rounds", type=int, default=6, help="rounds before the accuracy test")
    ap.add_argument("--precision", default="fp32", choices=["fp32", "bf16"])
    args = ap.parse_args()
    from ddl25spring_amd.data.images import DeviceImageDataset, load_images
    from ddl25spring_amd.data.split import split
    from ddl25spring_amd.fl.algorithms import FedAvg
    from ddl25spring_amd.fl.attacks import make_attack
    from ddl25spring_amd.models import mnist_cnn, resnet18_cifar
    from ddl25spring_amd.runtime import dist as rdist
    ctx = rdist.init()
    kind = "cifar10" if args.model == "resnet18" else "mnist"
    train = load_images(kind, True, args.train_size)
    test = load_images(kind, False, 2000)
    parts = split(8, True, 0, labels=train.labels)
    data, tdata = DeviceImageDataset(train, ctx.device), DeviceImageDataset(test, ctx.device)
    results = {}

    def build(groups):
        if args.model == "resnet18":
            return resnet18_cifar(10, groups=groups, precision=args.precision)
        return mnist_cnn(groups=groups, precision=args.precision)

    def make(agg, attacked):
        fa = FedAvg(build, data, parts,
                    lr=0.01, batch_size=100, client_fraction=1.0, seed=0, test_data=tdata,
                    aggregator=agg, agg_kwargs={"trim": 0.25, "f": 2}, ctx=ctx, eval_every=0)
        if attacked:
            # clients 0,1 flip labels (data poisoning), clients 2,3 flip (and scale) their update
            # signs (model poisoning): 4 of 8 clients hostile
            fa.attack = _Both(make_attack("sign_flip", [2, 3]), make_attack("label_flip", [0, 1]))
        return fa

    for agg in args.aggregators.split(","):
        fa = make(agg, True)
        for _ in range(args.warmup):
            fa.round()
        fa.timer.summary()
        times, agg_ms = [], []
        for _ in range(args.steps):
            dt, _ = fa.round()
            times.append(dt)
            agg_ms.append(fa.timer.summary().get("aggregate", float("nan")))
        res = {"rounds_per_s": round(len(times) / sum(times), 4),
               "aggregate_ms": round(float(np.mean(agg_ms)), 3)}
        if args.eval:
            for _ in range(args.acc_rounds - args.warmup - args.steps):
                fa.round()
            res["test_accuracy_attacked"] = round(fa.test(), 4)
            clean = make(agg, False)
            for _ in range(args.acc_rounds):
                clean.round()
            res["test_accuracy_clean"] = round(clean.test(), 4)
            del clean
        results[agg] = res
        del fa
    emit(ctx, metric="Byzantine-robust FedAvg rounds/s (8 clients, 2 label-flip + 2 sign-flip)",
         value=results.get("krum", next(iter(results.values())))["rounds_per_s"], unit="rounds/s",
         n_gpus=ctx.world, steps=args.steps, warmup=args.warmup, higher_is_better=True,
         scaling="strong", vs_baseline=None, dtype=args.precision, data="synthetic",
         acc_rounds=args.acc_rounds if args.eval else None, per_aggregator=results,
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
