"""Checkpoint / resume of a federated run (the reference keeps state only in memory).

``save(server, path, result)`` writes the server state (global model, round counter, RNG streams)
plus the RunResult so far, with tensors and plain containers only, so ``load`` uses
``torch.load(weights_only=True)`` — no pickled code. Only rank 0 writes; every rank loads the same
file, so a resumed multi-GPU run continues identically to an uninterrupted one.
"""
from __future__ import annotations

import dataclasses
import os

import torch

from .result import RunResult


def save(server, path: str, result: RunResult | None = None) -> None:
    if getattr(server.ctx, "rank", 0) != 0:
        return
    sd = {"server": server.state_dict()}
    if result is not None:
        sd["result"] = dataclasses.asdict(result)
    tmp = f"{path}.tmp"
    torch.save(sd, tmp)
    os.replace(tmp, path)  # atomic: a crash never leaves a torn checkpoint


def load(server, path: str) -> RunResult | None:
    sd = torch.load(path, map_location="cpu", weights_only=True)
    server.load_state_dict(sd["server"])
    if "result" in sd:
        return RunResult(**sd["result"])
    return None


def run_with_checkpoints(server, nr_rounds: int, path: str, every: int = 1) -> RunResult:
    """Run (or resume) ``nr_rounds`` rounds total, checkpointing every ``every`` rounds."""
    res = load(server, path) if os.path.exists(path) else None
    if res is None:
        res = RunResult(server.name, server.N, server.C, server.B, server.E, server.lr, server.seed)
    while server.round_idx < nr_rounds:
        part = server.run(1)
        for f in ("wall_time", "round_time", "samples", "message_count", "test_accuracy"):
            vals = getattr(part, f)
            if f == "wall_time" and getattr(res, f):
                vals = [round(res.wall_time[-1] + v, 1) for v in vals]
            getattr(res, f).extend(vals)
        if server.round_idx % every == 0 or server.round_idx == nr_rounds:
            save(server, path, res)
    return res
