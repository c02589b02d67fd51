"""Pipeline-parallel executor (naive / GPipe / 1F1B) over torch.distributed point-to-point.

Replaces the reference's hand-written per-rank send/recv choreographies
(lab/tutorial_1b/PP/1F1B/intro_PP_1F1B.py, intro_PP_1F1B_MB.py, intro_PP_1F1B_MP.py):
  * the schedule comes from the verified schedule IR (:mod:`.schedule`), so every stage posts
    matching sends/receives in a deadlock-free order;
  * activations / gradients stay on the GPU (RCCL ``send/recv`` over xGMI; the reference staged
    every message through host memory with ``.to("cpu")``);
  * a posted comm group is issued as ONE ``batch_isend_irecv`` (grouped P2P); over gloo (ranks that
    share a GPU, or CPU runs) device tensors are staged through host memory, since gloo's
    point-to-point moves CPU tensors only;
  * the loss is divided by the number of micro-batches (gradient averaging by loss scaling, as
    intro_PP_1F1B_MB.py:99 does), so an iteration equals one full-batch step.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from . import schedule as S


class PipelineStage:
    def __init__(self, module: torch.nn.Module, stage: int, n_stages: int, ranks: list[int] | None = None,
                 act_shape=None, act_dtype=None, device=None, group=None):
        """``ranks[s]`` = global rank of stage s in this pipeline (default: range(n_stages))."""
        self.module, self.stage, self.S = module, stage, n_stages
        self.ranks = ranks or list(range(n_stages))
        self.act_shape, self.act_dtype = act_shape, act_dtype
        self.device = device or next(module.parameters()).device
        self.group = group
        self.host_staged = torch.device(self.device).type == "cuda" and dist.is_initialized() and \
            dist.get_backend(group) == "gloo"

    @property
    def is_first(self):
        return self.stage == 0

    @property
    def is_last(self):
        return self.stage == self.S - 1

    def _p2p(self, ops):
        if not ops:
            return
        if not self.host_staged:
            for r in dist.batch_isend_irecv(ops):
                r.wait()
            return
        staged, back = [], []
        for op in ops:
            t = op.tensor
            if op.op is dist.isend:
                h = t.detach().cpu()
            else:
                h = torch.empty(t.shape, dtype=t.dtype)
                back.append((t, h))
            staged.append(dist.P2POp(op.op, h, op.peer, op.group))
        for r in dist.batch_isend_irecv(staged):
            r.wait()
        for t, h in back:
            t.copy_(h)

    def run(self, kind: str, n_micro: int, inputs=None, targets=None, loss_fn=None, grad_sync=None):
        """One training iteration (forward + backward of all micro-batches; no optimizer step).

        inputs: stage-0 micro-batch list; targets: last-stage micro-batch list.
        grad_sync: optional DP bucketer; its all-reduces only fire on the stage's LAST backward
        (earlier micro-batches accumulate under ``no_sync``).
        Returns the summed (already 1/M-scaled) loss on the last stage, else None."""
        import contextlib
        acts = S.make(kind, self.S, n_micro)
        prog = S.stage_program(acts, self.stage)
        last_bwd = max(i for i, st in enumerate(prog) if st[0].op == S.BWD)
        x_in, y_out, grads_in = {}, {}, {}
        total = None
        for si, step in enumerate(prog):
            ops, posted = [], []
            sync_ctx = contextlib.nullcontext()
            if grad_sync is not None and step[0].op == S.BWD and si != last_bwd:
                sync_ctx = grad_sync.no_sync()
            with sync_ctx:
                self._exec_step(step, ops, posted, x_in, y_out, grads_in, inputs, targets, loss_fn,
                                n_micro)
            if self.is_last:
                for a in step:
                    if a.op == S.FWD:
                        l = y_out[a.mb].detach()
                        total = l if total is None else total + l
            self._p2p(ops)
            for a, buf in posted:
                if a.op == S.RECV_ACT:
                    x_in[a.mb] = buf.requires_grad_(True)
                else:
                    grads_in[a.mb] = buf
        return total

    def _exec_step(self, step, ops, posted, x_in, y_out, grads_in, inputs, targets, loss_fn, n_micro):
        if True:
            for a in step:
                peer = self.ranks[a.peer] if a.peer >= 0 else -1
                if a.op == S.FWD:
                    if self.is_first:
                        inp = inputs[a.mb]
                    else:
                        inp = x_in[a.mb]
                    out = self.module(inp)
                    if self.is_last:
                        y_out[a.mb] = loss_fn(out, targets[a.mb]) / n_micro
                    else:
                        y_out[a.mb] = out
                elif a.op == S.BWD:
                    out = y_out.pop(a.mb)
                    if self.is_last:
                        out.backward()
                    else:
                        out.backward(grads_in.pop(a.mb))
                    if self.is_first:
                        x_in.pop(a.mb, None)
                elif a.op == S.SEND_ACT:
                    ops.append(dist.P2POp(dist.isend, y_out[a.mb].detach().contiguous(), peer, self.group))
                elif a.op == S.RECV_ACT:
                    buf = torch.empty(self.act_shape, dtype=self.act_dtype, device=self.device)
                    ops.append(dist.P2POp(dist.irecv, buf, peer, self.group))
                    posted.append((a, buf))
                elif a.op == S.SEND_GRAD:
                    g = x_in.pop(a.mb).grad
                    ops.append(dist.P2POp(dist.isend, g.contiguous(), peer, self.group))
                elif a.op == S.RECV_GRAD:
                    buf = torch.empty(self.act_shape, dtype=self.act_dtype, device=self.device)
                    ops.append(dist.P2POp(dist.irecv, buf, peer, self.group))
                    posted.append((a, buf))


def grid_ranks(rank: int, dp: int, pp: int):
    """2-D DP x PP grid (pipeline-major like the reference: pipeline_id = rank // pp,
    stage = rank % pp; DP groups = same stage across pipelines, e.g. {0,3},{1,4},{2,5})."""
    pipe, stage = divmod(rank, pp)
    pipe_ranks = [pipe * pp + s for s in range(pp)]
    dp_ranks = [p * pp + stage for p in range(dp)]
    return pipe, stage, pipe_ranks, dp_ranks
