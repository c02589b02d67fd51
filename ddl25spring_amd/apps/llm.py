"""LLaMA training over a DP x PP grid — the tutorial_1b scripts as one configurable program.

Covers, with one code path (reference lab/tutorial_1b):
  * intro.py                      dp=1 pp=1
  * DP/gradient_aggr/intro_DP_GA  dp=W, dp_mode="ga"  (bucketed all-reduce overlapped with backward)
  * DP/weight_aggr/intro_DP_WA    dp=W, dp_mode="wa"  (averaged weights written back — fixes Q1)
  * PP/1F1B/intro_PP_1F1B(_MB)    pp=W, schedule naive | gpipe | 1f1b, micro-batches
  * PP/1F1B/intro_PP_1F1B_MP      dp x pp grid (collective group creation; verified schedule)
Rank layout: rank = pipe * pp + stage. Every rank of a pipeline reads the same token stream
(``skip = pipe * 3000`` as the reference), so the last stage has its targets without extra
messages; stage weights start identical across pipelines (seeded init + broadcast).
"""
from __future__ import annotations

import os
import time
from dataclasses import asdict, dataclass

import torch

from ..data.text import SPTokenizer, TinyStories
from ..models.llama import LLama, causalLLMLoss, split_stages
from ..parallel.dp import GradBucketer, average_weights, broadcast_parameters
from ..parallel.pipeline import PipelineStage, grid_ranks, pipeline_links
from ..runtime.checkpoint import ShardedCheckpoint, load_optimizer_state, optimizer_state
from ..runtime.graphs import CAPTURE_MODE


@dataclass
class LLMConfig:
    vocab_size: int = 32000
    dmodel: int = 288
    num_heads: int = 6
    n_layers: int = 6
    ctx_size: int = 256
    batch_size: int = 3
    micro_batches: int = 1
    dp: int = 1
    pp: int = 1
    schedule: str = "1f1b"
    dp_mode: str = "ga"
    iters: int = 100
    lr: float = 8e-4
    seed: int = 0
    bucket_mb: float = 25.0
    log_every: int = 10
    fused_adam: bool = True
    graph: bool = True  # dp = pp = 1 on a GPU: replay the whole step (fwd, bwd, Adam) as a HIP graph
    ckpt_dir: str = ""  # sharded checkpoint directory (runtime/checkpoint.py); resumes if committed
    ckpt_every: int = 0  # commit a checkpoint every N optimizer steps (0: only at the end)
    # "fp32": the reference's precision (fp32 activations, stage messages and math; deterministic
    # kernels) — the default; "bf16": bf16 activations / MFMA operands with fp32 master weights
    precision: str = "fp32"


_RUN_FIELDS = ("vocab_size", "dmodel", "num_heads", "n_layers", "ctx_size", "batch_size",
               "micro_batches", "dp", "pp", "dp_mode", "lr", "seed", "fused_adam", "precision")


def _run_tag(cfg: "LLMConfig") -> str:
    """What a checkpoint must agree on to be resumable (not iters / logging / schedule)."""
    return ",".join(f"{k}={getattr(cfg, k)}" for k in _RUN_FIELDS)


class _PinnedH2D:
    """Token batches to the device without a host<->device sync: two pinned staging buffers used
    alternately, each refilled only after the copy that last read it has completed (a pageable
    copy would make the host wait for the GPU to drain, so it could not queue the next step)."""

    def __init__(self, shape, dtype, device):
        self.bufs = [torch.empty(shape, dtype=dtype).pin_memory() for _ in range(2)]
        self.events = [None, None]
        self.i, self.device = 0, device

    def __call__(self, x):
        i = self.i
        self.i ^= 1
        if self.events[i] is not None:
            self.events[i].synchronize()
        self.bufs[i].copy_(x)
        out = self.bufs[i].to(self.device, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self.events[i] = ev
        return out


def train_llm(cfg: LLMConfig, ctx, log=print, warmup: int = 0) -> dict:
    """Runs ``warmup`` untimed + ``cfg.iters`` timed iterations; returns losses and throughput.

    With ``cfg.ckpt_dir`` every rank checkpoints its own stage shard (weights, Adam moments, step)
    every ``cfg.ckpt_every`` steps and at the end, and a restarted job resumes from the last
    committed step: the token stream is re-positioned to that step, so a resumed run is
    bit-identical to an uninterrupted one (tests/test_checkpoint_cpu.py)."""
    if ctx.world != cfg.dp * cfg.pp:
        raise ValueError(f"world {ctx.world} != dp {cfg.dp} x pp {cfg.pp}")
    dev = ctx.device
    pipe, stage, pipe_ranks, _ = grid_ranks(ctx.rank, cfg.dp, cfg.pp)
    dp_group = ctx.new_groups("dp", [[p * cfg.pp + s for p in range(cfg.dp)] for s in range(cfg.pp)])
    torch.manual_seed(cfg.seed)
    full = LLama(vocab_size=cfg.vocab_size, dmodel=cfg.dmodel, num_heads=cfg.num_heads,
                 n_layers=cfg.n_layers, ctx_size=cfg.ctx_size, precision=cfg.precision)
    mod = split_stages(full, cfg.pp)[stage].to(dev)
    if cfg.dp > 1:
        broadcast_parameters(mod, ctx, src=stage, group=dp_group)  # pipeline 0's stage s is rank s
    if dev.type == "cuda" and cfg.fused_adam:
        from ..optim import FlatAdam
        # one fused Adam launch (bf16: also refreshes the bf16 weight shadow the GEMMs read; fp32:
        # the kernels read the master weights); weight grads accumulate straight into the flat
        # grad buffer (or the DP buckets)
        opt = FlatAdam(mod.parameters(), lr=cfg.lr, fused=True, bf16_shadow=cfg.precision == "bf16")
    else:
        opt = torch.optim.Adam(mod.parameters(), lr=cfg.lr)
    # DP-GA buckets are slices of FlatAdam's own flat gradient buffer (no second copy)
    sync = GradBucketer(mod, ctx, group=dp_group, bucket_mb=cfg.bucket_mb,
                        flat=opt if hasattr(opt, "offsets") else None) \
        if cfg.dp > 1 and cfg.dp_mode == "ga" else None
    if cfg.batch_size % cfg.micro_batches:
        raise ValueError("batch_size must be divisible by micro_batches")
    mb = cfg.batch_size // cfg.micro_batches
    # stage messages in the compute precision (the reference ships fp32 micro-batch activations,
    # intro_PP_1F1B_MB.py:57)
    act_dtype = torch.bfloat16 if dev.type == "cuda" and cfg.precision == "bf16" else torch.float32
    # per-link communicators: asynchronous P2P overlapped with compute (DDL_PP_ASYNC=0: blocking)
    links = pipeline_links(cfg.dp, cfg.pp) if (cfg.pp > 1 and ctx.is_distributed
                                               and os.environ.get("DDL_PP_ASYNC", "1") != "0") else None
    ps = PipelineStage(mod, stage, cfg.pp, ranks=pipe_ranks, act_shape=(mb, cfg.ctx_size, cfg.dmodel),
                       act_dtype=act_dtype, device=dev, links=links) if cfg.pp > 1 else None
    ckpt = ShardedCheckpoint(cfg.ckpt_dir, ctx, tag=_run_tag(cfg)) if cfg.ckpt_dir else None
    done = 0  # optimizer steps already taken (warm-up steps included: they train too)
    restored = ckpt.load() if ckpt is not None else None
    if restored is not None:
        done, st = restored
        mod.load_state_dict(st["model"])
        load_optimizer_state(opt, st["opt"])
        if log:
            log(f"[pipe {pipe} stage {stage}] resumed from step {done}")
    stream = iter(TinyStories(SPTokenizer(cfg.vocab_size), cfg.batch_size, cfg.ctx_size,
                              skip=pipe * 3000 + done, seed=1234 + cfg.seed))
    h2d = _PinnedH2D((cfg.batch_size, cfg.ctx_size), torch.int64, dev) if dev.type == "cuda" else None
    losses = []

    use_graph = (cfg.graph and dev.type == "cuda" and cfg.dp == 1 and cfg.pp == 1
                 and hasattr(opt, "t_dev"))
    gstate: dict = {}

    def body(xd):  # one dp = pp = 1 step on a static input buffer (capturable: no host syncs)
        opt.zero_grad()
        loss = None
        for m in torch.chunk(xd, cfg.micro_batches):
            l = causalLLMLoss(mod(m), m, scale=1.0 / cfg.micro_batches)
            l.backward()
            loss = l.detach() if loss is None else loss + l.detach()
        opt.step()
        return loss

    def graph_step(xd):
        if not gstate:
            sx = xd.clone()
            # the warm-up steps really train: snapshot the optimizer state and restore it after
            # capture, so the first replay is exactly step 1
            snap = [t.clone() for t in (opt.data, opt.m, opt.v, opt.t_dev)]
            t_host = opt.t
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                for _ in range(2):
                    body(sx)
            torch.cuda.current_stream().wait_stream(side)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, capture_error_mode=CAPTURE_MODE):
                out = body(sx)
            for t, v in zip((opt.data, opt.m, opt.v, opt.t_dev), snap):
                t.copy_(v)
            opt.t = t_host
            opt.sync_shadow()
            gstate.update(g=g, x=sx, loss=out)
        gstate["x"].copy_(xd)
        gstate["g"].replay()
        opt.t += 1
        return gstate["loss"]

    def step():
        x = next(stream)
        x = h2d(x) if h2d is not None else x.to(dev)
        if use_graph:
            return graph_step(x)
        if sync is not None:
            sync.zero_grad()
        else:
            opt.zero_grad()
        if ps is None:
            loss = None
            mbs = torch.chunk(x, cfg.micro_batches)
            for i, m in enumerate(mbs):
                l = causalLLMLoss(mod(m), m, scale=1.0 / cfg.micro_batches)
                if sync is not None and i < len(mbs) - 1:
                    with sync.no_sync():
                        l.backward()
                else:
                    l.backward()
                loss = l.detach() if loss is None else loss + l.detach()
        else:
            mbs = list(torch.chunk(x, cfg.micro_batches))
            loss = ps.run(cfg.schedule, cfg.micro_batches, inputs=mbs, targets=mbs,
                          loss_fn=causalLLMLoss, grad_sync=sync)
        if sync is not None:
            sync.finish()
        opt.step()
        if cfg.dp > 1 and cfg.dp_mode == "wa":
            average_weights(mod, ctx, group=dp_group)
            if hasattr(opt, "sync_shadow"):
                opt.sync_shadow()
        return loss

    def save(n):
        if dev.type == "cuda":
            torch.cuda.synchronize()
        ckpt.save(n, {"model": mod.state_dict(), "opt": optimizer_state(opt)})

    total = warmup + cfg.iters
    while done < warmup:
        step()
        done += 1
    if dev.type == "cuda":
        torch.cuda.synchronize()
    ctx.barrier()
    t0 = time.perf_counter()
    timed = total - done
    while done < total:
        it = done - warmup
        loss = step()
        done += 1
        if loss is not None and (it % cfg.log_every == 0 or it == cfg.iters - 1):
            lv = float(loss)
            losses.append((it, lv))
            if log:
                log(f"[pipe {pipe} stage {stage}] iter {it} loss {lv:.4f}")
        if ckpt is not None and cfg.ckpt_every and done % cfg.ckpt_every == 0 and done < total:
            save(done)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    ctx.barrier()
    dt = ctx.max_scalar(time.perf_counter() - t0)
    if ckpt is not None and (restored is None or restored[0] < total):
        save(total)
    tokens = cfg.dp * cfg.batch_size * cfg.ctx_size * timed
    return {"losses": losses, "seconds": dt, "tokens_per_s": tokens / max(dt, 1e-9),
            "ms_per_iter": 1e3 * dt / max(1, timed), "config": asdict(cfg),
            "resumed_from": None if restored is None else restored[0]}
