"""Sharded, atomic checkpoint / resume for multi-rank jobs (LLM DP x PP grids, split-NN VFL).

The reference keeps all training state in memory (no checkpointing anywhere in
lab/tutorial_1b or lab/tutorial_3); a crashed 8-rank job restarts from step 0. Here every rank
writes its OWN shard (its pipeline stage's weights, its optimizer moments, its step counter) and
the job commits a step only when all shards are on disk:

    <dir>/step00000040/rank00003.pt     one shard per rank (torch.save of tensors / plain data)
    <dir>/latest.json                   {"step": 40, "world": 4, "tag": ...} — the commit record

1. every rank writes ``rank{r}.pt.tmp`` then renames it (a crash never leaves a torn shard);
2. barrier;
3. rank 0 rewrites ``latest.json`` atomically and prunes older step directories.

A job killed between 1 and 3 resumes from the previous committed step. Shards hold only tensors
and plain containers, so ``load`` uses ``torch.load(weights_only=True)`` — nothing in a checkpoint
is executed. Ranks only touch their own shard (no gather through rank 0): at 288 GB per GPU a
stage shard plus Adam moments is written at local-disk speed in parallel on every rank.
"""
from __future__ import annotations

import json
import os
import shutil

import torch


def _to_cpu(obj):
    if isinstance(obj, torch.Tensor):
        return obj.detach().to("cpu", copy=True)
    if isinstance(obj, dict):
        return {k: _to_cpu(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to_cpu(v) for v in obj)
    return obj


def optimizer_state(opt) -> dict:
    """Optimizer state as tensors + plain data: FlatAdam (flat data/m/v/step), the ParamStore
    optimizers, or any ``torch.optim`` optimizer (its own ``state_dict``)."""
    from ..optim import FlatAdam
    if isinstance(opt, FlatAdam):
        return {"kind": "flat_adam", "data": opt.data, "m": opt.m, "v": opt.v, "t": opt.t}
    if hasattr(opt, "state_dict"):
        return {"kind": "torch", "state": opt.state_dict()}
    raise TypeError(f"no checkpoint format for optimizer {type(opt).__name__}")


@torch.no_grad()
def load_optimizer_state(opt, sd: dict) -> None:
    from ..optim import FlatAdam
    if sd["kind"] == "flat_adam":
        if not isinstance(opt, FlatAdam):
            raise TypeError("checkpoint holds FlatAdam state; the optimizer is not a FlatAdam")
        for name in ("data", "m", "v"):
            dst, src = getattr(opt, name), sd[name]
            if dst.shape != src.shape:
                raise ValueError(f"FlatAdam.{name}: checkpoint {tuple(src.shape)} != {tuple(dst.shape)}")
            dst.copy_(src)
        opt.t = int(sd["t"])
        if opt.t_dev is not None:
            opt.t_dev.fill_(opt.t)
        opt.sync_shadow()
    else:
        opt.load_state_dict(sd["state"])


class ShardedCheckpoint:
    """One directory of step-tagged per-rank shards; see the module docstring."""

    def __init__(self, directory: str, ctx, tag: str = "", keep: int = 1):
        self.dir, self.ctx, self.tag, self.keep = directory, ctx, tag, max(1, keep)
        self.rank, self.world = getattr(ctx, "rank", 0), getattr(ctx, "world", 1)
        if self.rank == 0:
            os.makedirs(directory, exist_ok=True)

    def _step_dir(self, step: int) -> str:
        return os.path.join(self.dir, f"step{step:08d}")

    def _shard(self, step: int, rank: int) -> str:
        return os.path.join(self._step_dir(step), f"rank{rank:05d}.pt")

    def latest(self) -> int | None:
        """The last committed step (None: nothing committed). Every rank reads the same record."""
        try:
            with open(os.path.join(self.dir, "latest.json")) as f:
                rec = json.load(f)
        except FileNotFoundError:
            return None
        if rec.get("world") != self.world:
            raise ValueError(f"checkpoint in {self.dir} was written by {rec.get('world')} ranks, "
                             f"this job has {self.world}")
        if self.tag and rec.get("tag") != self.tag:
            raise ValueError(f"checkpoint tag {rec.get('tag')!r} != {self.tag!r} (different run config)")
        return int(rec["step"])

    def save(self, step: int, state: dict) -> None:
        """Collective: every rank calls it with its own ``state`` (tensors on any device)."""
        os.makedirs(self._step_dir(step), exist_ok=True)
        path = self._shard(step, self.rank)
        torch.save({"step": step, "rank": self.rank, "state": _to_cpu(state)}, path + ".tmp")
        os.replace(path + ".tmp", path)
        self.ctx.barrier()
        if self.rank == 0:
            rec = {"step": step, "world": self.world, "tag": self.tag}
            tmp = os.path.join(self.dir, "latest.json.tmp")
            with open(tmp, "w") as f:
                json.dump(rec, f)
            os.replace(tmp, os.path.join(self.dir, "latest.json"))
            steps = sorted(int(n[4:]) for n in os.listdir(self.dir)
                           if n.startswith("step") and n[4:].isdigit())
            for old in steps:
                if old < step and old not in steps[-self.keep:]:
                    shutil.rmtree(self._step_dir(old), ignore_errors=True)
        self.ctx.barrier()  # nobody races ahead and re-saves before the commit record is written

    def load(self, step: int | None = None) -> tuple[int, dict] | None:
        """This rank's shard of ``step`` (default: the latest committed step), or None."""
        step = self.latest() if step is None else step
        if step is None:
            return None
        sd = torch.load(self._shard(step, self.rank), map_location="cpu", weights_only=True)
        if sd["step"] != step or sd["rank"] != self.rank:
            raise ValueError(f"shard {self._shard(step, self.rank)} is for step {sd['step']} rank {sd['rank']}")
        return step, sd["state"]
