"""Shared bench plumbing: env rendezvous, timed loop (barrier + synchronize on both sides, max over
ranks), one JSON line from rank 0."""
from __future__ import annotations

import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(ctx, step, steps: int, warmup: int) -> float:
    """Seconds for ``steps`` calls of ``step`` after ``warmup`` untimed ones (max over ranks)."""
    for _ in range(warmup):
        step()
    if ctx.device.type == "cuda":
        torch.cuda.synchronize()
    ctx.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    if ctx.device.type == "cuda":
        torch.cuda.synchronize()
    ctx.barrier()
    return ctx.max_scalar(time.perf_counter() - t0)


def emit(ctx, **rec):
    if ctx.rank == 0:
        print(json.dumps(rec), flush=True)
