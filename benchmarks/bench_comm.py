"""Collective bandwidth sweep over the framework's communication layer (RCCL over xGMI on GPUs,
gloo on CPU): all-reduce, reduce-scatter, all-gather, all-to-all and broadcast, 4 KiB .. 256 MiB.

Every collective the framework issues goes through one of these calls: DP gradient
buckets and FedAvg weight averages (all-reduce, C3/C4/C11/C13), robust aggregation's coordinate
sharding (all-to-all + all-gather, C17), server -> client download (broadcast, C12). The sizes
that matter: FL MnistCnn rows 4.8 MB, ResNet-18 45 MB, ResNet-50 gradient buckets 64 MB.
``ipc_all_reduce`` is the peer-read all-reduce (runtime/ipc.py, one kernel over hipIPC-mapped
buffers); its curve against ``all_reduce`` (RCCL) sets ``DDL_IPC_MAX_BYTES``.

Reported per (op, size), rccl-tests conventions: algbw = bytes / t; busbw = algbw x factor with
factor 2(W-1)/W (all-reduce), (W-1)/W (reduce-scatter, all-gather, all-to-all), 1 (broadcast).
One JSON line per op with the full curve; rank 0 prints.

    python -m torch.distributed.run --nproc-per-node 8 benchmarks/bench_comm.py
"""
from __future__ import annotations

import argparse
import json

import torch
import torch.distributed as dist

from _common import timed


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--min-kb", type=int, default=4)
    ap.add_argument("--max-mb", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--ops", default="all_reduce,ipc_all_reduce,reduce_scatter,all_gather,all_to_all,"
                                     "broadcast")
    args = ap.parse_args()
    from ddl25spring_amd.runtime import dist as rdist
    ctx = rdist.init()
    W, dev = ctx.world, ctx.device
    sizes = []
    b = args.min_kb * 1024
    while b <= args.max_mb * 2 ** 20:
        sizes.append(b)
        b *= 4
    ipc = None
    if "ipc_all_reduce" in args.ops and ctx.is_distributed and dev.type == "cuda":
        from ddl25spring_amd.runtime.ipc import IpcAllReduce
        ipc = IpcAllReduce(ctx.rank, W, dev, capacity=min(args.max_mb, 64) * 2 ** 20)
    factor = {"all_reduce": 2 * (W - 1) / W, "ipc_all_reduce": 2 * (W - 1) / W,
              "reduce_scatter": (W - 1) / W,
              "all_gather": (W - 1) / W, "all_to_all": (W - 1) / W, "broadcast": 1.0}
    for op in args.ops.split(","):
        curve = []
        for nbytes in sizes:
            if op == "ipc_all_reduce" and (ipc is None or nbytes > ipc.cap):
                continue
            n = max(W, nbytes // 4 // W * W)  # fp32 elements, divisible by the world size
            x = torch.ones(n, dtype=torch.float32, device=dev)
            y = torch.empty_like(x)
            part = torch.empty(n // W, dtype=torch.float32, device=dev)
            if not ctx.is_distributed:
                fn = lambda: None  # noqa: E731  (one rank: nothing moves)
            elif op == "all_reduce":
                fn = lambda: dist.all_reduce(x)  # noqa: E731
            elif op == "ipc_all_reduce":
                fn = lambda: ipc.all_reduce(x)  # noqa: E731
            elif op == "reduce_scatter":
                fn = lambda: dist.reduce_scatter_tensor(part, x)  # noqa: E731
            elif op == "all_gather":
                fn = lambda: dist.all_gather_into_tensor(y, part)  # noqa: E731
            elif op == "all_to_all":
                fn = lambda: dist.all_to_all_single(y, x)  # noqa: E731
            elif op == "broadcast":
                fn = lambda: dist.broadcast(x, 0)  # noqa: E731
            else:
                raise ValueError(op)
            t = timed(ctx, fn, args.iters, args.warmup) / args.iters
            moved = n * 4
            algbw = moved / t / 1e9 if W > 1 else None
            curve.append({"bytes": moved, "us": round(t * 1e6, 1),
                          "algbw_GBps": None if algbw is None else round(algbw, 2),
                          "busbw_GBps": None if algbw is None else round(algbw * factor[op], 2)})
        if ctx.rank == 0 and curve:
            peak = max((c["busbw_GBps"] or 0.0) for c in curve)
            print(json.dumps({"metric": f"{op} bus bandwidth", "value": peak or None, "unit": "GB/s",
                              "n_gpus": W if dev.type == "cuda" else 0, "ranks": W,
                              "backend": dist.get_backend() if ctx.is_distributed else None,
                              "higher_is_better": True, "curve": curve}), flush=True)
    if ipc is not None:
        ipc.check()
        ipc.close()
    rdist.shutdown()


if __name__ == "__main__":
    main()
