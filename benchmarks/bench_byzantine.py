"""BASELINE config #4: Byzantine-robust FL — Krum / trimmed-mean / coordinate-median under
label-flip + sign-flip attackers, 8 clients (ResNet-18, CIFAR-10 shape, the headline workload).

Per aggregator: FedAvg rounds/s under attack over ``--steps`` (default 10) UNSYNCHRONISED rounds
(the host enqueues round r+1 while the GPU runs round r, as bench.py's headline does; one device
sync brackets the timed span), the device time of the aggregation phase (coordinate-sharded
all-to-all + bitonic selection / fp32-MFMA Gram kernels) from two extra synchronised rounds, the
same rounds/s of the CLEAN mean run (no attacker) as the yardstick, and the robustness itself:
test accuracy after ``--acc-rounds`` rounds on the learnable synthetic CIFAR set, clean (no
attacker) vs attacked, for every aggregator (``--no-eval`` skips the accuracy runs).
"""
from __future__ import annotations

import argparse

import numpy as np

from _common import emit


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10, help="timed (unsynchronised) rounds per aggregator")
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--model", default="resnet18")
    ap.add_argument("--train-size", type=int, default=50000)
    ap.add_argument("--aggregators", default="mean,median,trimmed_mean,krum")
    ap.add_argument("--no-eval", dest="eval", action="store_false")
    ap.add_argument("--acc-rounds", type=int, default=16,
                    help="rounds before the accuracy test (at least the timed run's rounds)")
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

    import time

    import torch

    def timed(fa):
        """rounds/s over args.steps unsynchronised rounds (max over ranks), then the aggregation
        phase's device time from 2 synchronised rounds."""
        for _ in range(args.warmup):
            fa.round()
        fa.sync_rounds = False
        if ctx.device.type == "cuda":
            torch.cuda.synchronize()
        ctx.barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            fa.round()
        if ctx.device.type == "cuda":
            torch.cuda.synchronize()
        ctx.barrier()
        dt = ctx.max_scalar(time.perf_counter() - t0)
        fa.sync_rounds = True
        fa.timer.summary()
        agg_ms = []
        for _ in range(2):
            fa.round()
            agg_ms.append(fa.timer.summary().get("aggregate", float("nan")))
        return args.steps / dt, float(np.mean(agg_ms))

    clean_rps = None
    if "mean" in args.aggregators.split(","):
        fa = make("mean", False)
        clean_rps, _ = timed(fa)
        del fa
        if ctx.rank == 0:
            import sys
            print(f"[bench_byzantine] clean mean: {clean_rps:.4f} rounds/s", file=sys.stderr, flush=True)
    for agg in args.aggregators.split(","):
        fa = make(agg, True)
        rps, agg_ms = timed(fa)
        res = {"rounds_per_s": round(rps, 4), "aggregate_ms": round(agg_ms, 3)}
        if clean_rps:
            res["vs_clean_mean"] = round(rps / clean_rps, 4)
        if args.eval:
            total = max(args.acc_rounds, fa.round_idx)
            while fa.round_idx < total:
                fa.round()
            res["test_accuracy_attacked"] = round(fa.test(), 4)
            clean = make(agg, False)
            for _ in range(total):
                clean.round()
            res["test_accuracy_clean"] = round(clean.test(), 4)
            del clean
        results[agg] = res
        if ctx.rank == 0:  # progress (a full sweep runs for minutes)
            import sys
            print(f"[bench_byzantine] {agg}: {res}", file=sys.stderr, flush=True)
        del fa
    emit(ctx, metric="Byzantine-robust FedAvg rounds/s (8 clients, 2 label-flip + 2 sign-flip)",
         value=results.get("krum", next(iter(results.values())))["rounds_per_s"], unit="rounds/s",
         n_gpus=ctx.world, steps=args.steps, warmup=args.warmup, higher_is_better=True,
         scaling="strong", vs_baseline=None, dtype=args.precision, data="synthetic",
         acc_rounds=max(args.acc_rounds, args.warmup + args.steps + 2) if args.eval else None,
         per_aggregator=results,
         clean_mean_rounds_per_s=None if clean_rps is None else round(clean_rps, 4),
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
