"""Headline benchmark: FedAvg rounds/s + local samples/s, ResNet-18, CIFAR-10 shape, 8 clients.

BASELINE.json config #2 ("Horizontal FedAvg ResNet-18, CIFAR-10-shape, 8 IID clients = 8 x
MI355X"). One *step* = one full FedAvg round: every one of the 8 clients runs E=1 local epoch of
mini-batch SGD (B=100, lr=0.01 — the reference's FedAvg defaults, homework-1.ipynb:50-59) over its
IID shard of the 50,000-image CIFAR-10-shaped training set (6,250 images each), then the server
takes the n_k-weighted average (RCCL all-reduce across GPUs). Total work is fixed (8 clients) and
spread over N GPUs, i.e. strong scaling: at N=1 the 8 clients run client-batched on one GPU, at N=8
each GPU is one client.

Data: synthetic CIFAR-10-shaped uint8 images (learnable class templates), random-init weights.
Precision (``--precision``, default fp32 = the reference's, lab/tutorial_1a/hfl_complete.py:39-80):
  fp32 — activations, weights, gradients and BN in fp32 end to end (bn_f32.hip). The convs run
         the X6 engine by default (``fp32_conv_math`` "auto"): every fp32 operand split exactly
         into three bf16 pieces, the six piece products above one fp32 rounding on the bf16 MFMA
         (conv_x6h.hip: halo-staged FWD / stride-1 DGRAD; conv_f32.hip: the rest), or the exact
         fp32 MFMA where the tuner measured that faster; both meet the fp32 tolerances of
         tests/test_fp32_gpu.py. The step is bitwise deterministic, so the JSON line also
         carries a sha256 of the final server weights (``w_global_sha256``);
  bf16 — bf16 MFMA operands / activations with fp32 master weights, grads, BN statistics and
         aggregation (conv_igemm.hip), the faster non-reference-precision mode.

    python bench.py --gpus 1 --steps 3 --warmup 1
    torchrun --nproc-per-node 8 bench.py --gpus 8 ...
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

import torch

METRIC = "FedAvg rounds/sec + local samples/sec, ResNet-18 CIFAR-10-shape, 8 clients"
# the reference publishes no throughput; the number to beat is the reference's own FedAvg
# loop (hfl_complete.py FedAvgServer: per-client nn.Module replicas, host-staged weights, fp32) on
# the same config, timed on one MI355X with stock PyTorch-ROCm (benchmarks/bench_reference_eager.py
# --variant faithful; profiles/reference_eager_r3.jsonl).
REFERENCE_SAMPLES_PER_S = {"fp32": 5296.8}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3, help="timed FedAvg rounds")
    ap.add_argument("--warmup", type=int, default=1, help="untimed FedAvg rounds")
    ap.add_argument("--clients", type=int, default=8)
    ap.add_argument("--batch", type=int, default=100)
    ap.add_argument("--epochs", type=int, default=1)
    ap.add_argument("--lr", type=float, default=0.01)
    ap.add_argument("--train-size", type=int, default=50000)
    ap.add_argument("--model", default="resnet18")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--sync-rounds", action="store_true",
                    help="synchronise host and device around every timed round (A/B)")
    ap.add_argument("--eval", action="store_true", help="also report test accuracy (untimed)")
    ap.add_argument("--backend", default=None,
                    help="collective backend (default: nccl = RCCL on GPUs); gloo lets several "
                         "ranks share one GPU for a functional rehearsal")
    ap.add_argument("--precision", default="fp32", choices=("fp32", "bf16"),
                    help="compute precision (fp32 = the reference's; bf16 = bf16 MFMA / activations)")
    ap.add_argument("--deterministic", action="store_true",
                    help="require a bitwise-reproducible run (the fp32 path: no float atomics; two runs "
                         "print the same w_global_sha256)")
    args = ap.parse_args()
    if args.deterministic and args.precision != "fp32":
        ap.error("--deterministic needs --precision fp32 (the bf16 path reduces with float atomics)")

    from ddl25spring_amd.runtime import dist as rdist
    ctx = rdist.init(backend=args.backend)
    if ctx.device.type != "cuda":
        print("bench.py needs a GPU", file=sys.stderr)
        rdist.shutdown()
        sys.exit(2)
    from ddl25spring_amd.data.images import DeviceImageDataset, synthetic_images
    from ddl25spring_amd.data.split import split
    from ddl25spring_amd.fl.algorithms import FedAvg
    from ddl25spring_amd.models import resnet18_cifar

    train = synthetic_images("cifar10", args.train_size, seed=0)
    test = synthetic_images("cifar10", 2000, seed=1) if args.eval else None
    dtrain = DeviceImageDataset(train, ctx.device)
    dtest = DeviceImageDataset(test, ctx.device) if test is not None else None
    parts = split(args.clients, True, 10, labels=train.labels)
    base_fn = {"resnet18": resnet18_cifar}[args.model]

    def model_fn(groups):
        return base_fn(10, groups=groups, precision=args.precision)
    fl = FedAvg(model_fn, dtrain, parts, lr=args.lr, batch_size=args.batch,
                local_epochs=args.epochs, client_fraction=1.0, seed=10, test_data=dtest,
                use_graph=not args.no_graph, eval_every=0)

    for _ in range(args.warmup):
        fl.round()
    # timed rounds without per-round host <-> device syncs: the host plans and enqueues round r+1
    # while the GPU runs round r (FederatedBase.sync_rounds); the work per round is unchanged
    fl.sync_rounds = args.sync_rounds
    ctx.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    samples = 0
    for _ in range(args.steps):
        _, s = fl.round()
        samples += s
    ctx.barrier()
    torch.cuda.synchronize()
    elapsed = ctx.max_scalar(time.perf_counter() - t0)
    if not fl.sync_rounds:
        samples = int(ctx.sum_scalar(samples))  # round() returned this rank's samples
        fl.sync_rounds = True
    ms_per_round = 1000.0 * elapsed / args.steps
    samples_per_s = samples / elapsed
    rounds_per_s = args.steps / elapsed
    acc = fl.test() if args.eval else None
    w_hash = hashlib.sha256(fl.w_global.detach().cpu().numpy().tobytes()).hexdigest()
    hashes = [w_hash]
    if ctx.world > 1:  # the replicated server model: every rank must hold the same bits
        import torch.distributed as tdist
        hashes = [None] * ctx.world
        tdist.all_gather_object(hashes, w_hash)
    from ddl25spring_amd.ops import functional_f32 as F32
    ref = REFERENCE_SAMPLES_PER_S.get(args.precision)
    if ctx.is_main:
        out = {
            "metric": METRIC,
            "value": round(samples_per_s, 1),
            "unit": "samples/s",
            "n_gpus": ctx.world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_round, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": round(samples_per_s / ref, 2) if ref else None,
            "baseline": ({"value": ref, "unit": "samples/s", "what": "reference FedAvg loop (hfl_complete.py), "
                          "stock PyTorch-ROCm fp32, 1x MI355X"} if ref else None),
            "dtype": args.precision,
            "data": "synthetic",
            "w_global_sha256": w_hash,
            "rounds_per_sec": round(rounds_per_s, 4),
            "local_samples_per_round": samples // max(args.steps, 1),
            "config": {"model": "resnet18-cifar10", "global_batch": args.batch * args.clients,
                       "seq_len": None, "parallelism": f"fedavg-{args.clients}clients-dp{ctx.world}",
                       "clients": args.clients, "local_batch": args.batch,
                       "local_epochs": args.epochs, "lr": args.lr,
                       "samples_per_client": args.train_size // args.clients,
                       "client_slots_per_gpu": fl.slots, "hip_graphs": not args.no_graph,
                       "fp32_conv_math": F32.math() if args.precision == "fp32" else None},
        }
        if ctx.world > 1:
            wb = fl.w_global.numel() * 4
            # the round's cross-rank weight reduction (fl/aggregate.py) and the all-reduce path the
            # context's policy picks for a message of that size (runtime/dist.py)
            agg = fl.aggregator.describe(ctx) if hasattr(fl.aggregator, "describe") else \
                type(fl.aggregator).__name__
            out["aggregation"] = agg
            # the transport of the round's weight reduction: the IPC peer-read kernel (rank-ordered
            # sum), an all-gather, or -- only for the unordered mean -- the all-reduce path the
            # context's size policy picks for a message of that size
            comm = {"weights_bytes": wb, "backend": ctx.backend, **ctx.ipc_policy}
            if agg == "all-reduce":
                comm["allreduce_path"] = rdist.allreduce_path(ctx, wb)
            else:
                comm["transport"] = "ipc" if agg.startswith("ipc") else "all_gather"
            out["comm"] = comm
            out["rank_hashes_equal"] = len(set(hashes)) == 1
        if args.precision == "fp32":
            # the X6 engine's chain lengths (zero-start MFMA chains before each IEEE add, docs/KERNELS.md
            # "Chain length"); the measured gradient error of this tree: profiles/fp32_grad_accuracy_r6.txt
            # (scripts/debug_r18_grads.py); no accuracy figure is hard-coded here
            out["fp32_chains"] = {"x6h_tap_steps": 3, "x6hw_pixel_steps": 2}
        if acc is not None:
            out["test_accuracy"] = acc
        print(json.dumps(out), flush=True)
    rdist.shutdown()


if __name__ == "__main__":
    main()
