"""Pipeline-parallel executor (naive / GPipe / 1F1B) over torch.distributed point-to-point.

Replaces the reference's hand-written per-rank send/recv choreographies
(lab/tutorial_1b/PP/1F1B/intro_PP_1F1B.py, intro_PP_1F1B_MB.py, intro_PP_1F1B_MP.py):
  * the schedule comes from the verified schedule IR (:mod:`.schedule`), so every stage posts
    matching sends/receives in a deadlock-free order;
  * activations / gradients stay on the GPU (RCCL ``send/recv`` over xGMI; the reference staged
    every message through host memory with ``.to("cpu")``);
  * with per-link communicators (``pipeline_links``: one process group per DIRECTED stage link,
    activations s -> s+1 and gradients s+1 -> s apart) the P2P is asynchronous and overlaps
    compute: the receives of the next comm step are posted BEFORE the current compute step, sends
    are posted right after the compute that produced them, and a stage waits for a received tensor
    only when a compute step consumes it (``work.wait()``: on RCCL a device-side stream wait, the
    host keeps queueing). Each link's stream carries one direction between one pair of ranks in
    schedule order, so posting receives early cannot create a send/recv cycle on a shared stream;
    the link communicators are initialised up front in one global order (no lazy-init rendezvous
    inside the schedule). Without links the legacy path posts each comm group as ONE blocking
    ``batch_isend_irecv``;
  * over gloo (ranks that share a GPU, or CPU runs) device tensors are staged through host memory,
    since gloo's point-to-point moves CPU tensors only;
  * the loss is divided by the number of micro-batches (gradient averaging by loss scaling, as
    intro_PP_1F1B_MB.py:99 does), so an iteration equals one full-batch step.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from . import schedule as S


class PipelineStage:
    def __init__(self, module: torch.nn.Module, stage: int, n_stages: int, ranks: list[int] | None = None,
                 act_shape=None, act_dtype=None, device=None, group=None, links: dict | None = None):
        """``ranks[s]`` = global rank of stage s in this pipeline (default: range(n_stages)).
        ``links``: ``pipeline_links(...)`` (every rank's dict, built collectively) -> asynchronous,
        compute-overlapped P2P; None -> blocking grouped P2P on ``group``."""
        self.module, self.stage, self.S = module, stage, n_stages
        self.ranks = ranks or list(range(n_stages))
        self.act_shape, self.act_dtype = act_shape, act_dtype
        self.device = device or next(module.parameters()).device
        self.group = group
        self.host_staged = torch.device(self.device).type == "cuda" and dist.is_initialized() and \
            dist.get_backend(group) == "gloo"
        self.links = None
        if links is not None and dist.is_initialized():
            me = self.ranks[stage]
            self.links = {k: g for k, g in links.items() if me in k}
            self.link_host_staged = torch.device(self.device).type == "cuda" and any(
                dist.get_backend(g) == "gloo" for g in self.links.values())
            _warm_links(links, me, self.device)

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
        if self.links is not None:
            return self._run_async(kind, n_micro, inputs, targets, loss_fn, grad_sync)
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

    # ------------------------------------------------------------------ asynchronous (per-link) P2P
    # One communicator per DIRECTED stage link (pipeline_links): a stage posts the receives of the
    # comm steps that follow BEFORE it computes, and its sends complete in the background, while the
    # DP gradient bucketer's all-reduces run on other communicators. Nothing orders these kernels
    # across ranks, so with RCCL this relies on the GPU co-scheduling them (each collective kernel
    # occupies a few CUs and spins until its peers arrive; a GPU that could not keep a posted
    # receive and another link's kernel resident at once could deadlock). On MI355X the kernels are
    # small next to 256 CUs; DDL_PP_ASYNC=0 (apps/llm.py builds no links) selects the grouped,
    # step-ordered batch_isend_irecv path of ``run`` as the fallback. Covered on gloo by
    # tests/test_parallel_cpu.py::test_dp_x_pp_grid_runs_and_replicas_agree[3] (dp 2 x pp 3 + bucketer).
    def _link(self, op: int, peer_stage: int):
        me, peer = self.ranks[self.stage], self.ranks[peer_stage]
        return self.links[(me, peer) if op in (S.SEND_ACT, S.SEND_GRAD) else (peer, me)], peer

    def _post_recv(self, a, pending):
        if (a.op, a.mb) in pending:
            return
        g, peer = self._link(a.op, a.peer)
        buf = torch.empty(self.act_shape, dtype=self.act_dtype,
                          device="cpu" if self.link_host_staged else self.device)
        pending[(a.op, a.mb)] = (dist.irecv(buf, peer, group=g), buf)

    def _take(self, pending, op, mb):
        work, buf = pending.pop((op, mb))
        work.wait()  # RCCL: the current stream waits for the receive; the host does not block
        return buf.to(self.device) if self.link_host_staged else buf

    def _post_send(self, a, t, sends):
        g, peer = self._link(a.op, a.peer)
        t = t.detach().contiguous()
        if self.link_host_staged:
            t = t.cpu()
        sends.append((dist.isend(t, peer, group=g), t))  # keep the tensor alive until completion

    def _run_async(self, kind, n_micro, inputs, targets, loss_fn, grad_sync):
        import contextlib
        prog = S.stage_program(S.make(kind, self.S, n_micro), self.stage)
        last_bwd = max(i for i, st in enumerate(prog) if st[0].op == S.BWD)
        pending, sends = {}, []
        x_in, y_out = {}, {}
        total = None
        for si, step in enumerate(prog):
            a0 = step[0]
            if a0.op not in (S.FWD, S.BWD):  # a comm step: receives (unless posted early), then sends
                for a in step:
                    if a.op in (S.RECV_ACT, S.RECV_GRAD):
                        self._post_recv(a, pending)
                for a in step:
                    if a.op == S.SEND_ACT:
                        self._post_send(a, y_out[a.mb], sends)
                    elif a.op == S.SEND_GRAD:
                        self._post_send(a, x_in.pop(a.mb).grad, sends)
                continue
            # post the receives of the comm steps that follow BEFORE this compute step
            j = si + 1
            while j < len(prog) and prog[j][0].op not in (S.FWD, S.BWD):
                for a in prog[j]:
                    if a.op in (S.RECV_ACT, S.RECV_GRAD):
                        self._post_recv(a, pending)
                j += 1
            sync_ctx = contextlib.nullcontext()
            if grad_sync is not None and a0.op == S.BWD and si != last_bwd:
                sync_ctx = grad_sync.no_sync()
            with sync_ctx:
                if a0.op == S.FWD:
                    if self.is_first:
                        inp = inputs[a0.mb]
                    else:
                        inp = self._take(pending, S.RECV_ACT, a0.mb).requires_grad_(True)
                        x_in[a0.mb] = inp
                    out = self.module(inp)
                    if self.is_last:
                        l = loss_fn(out, targets[a0.mb]) / n_micro
                        y_out[a0.mb] = l
                        total = l.detach() if total is None else total + l.detach()
                    else:
                        y_out[a0.mb] = out
                else:
                    out = y_out.pop(a0.mb)
                    if self.is_last:
                        out.backward()
                    else:
                        out.backward(self._take(pending, S.RECV_GRAD, a0.mb))
                    if self.is_first:
                        x_in.pop(a0.mb, None)
        for work, _ in sends:
            work.wait()
        assert not pending, f"unconsumed receives {sorted(pending)}"
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


def pipeline_links(dp: int, pp: int) -> dict | None:
    """One process group per DIRECTED stage link of every pipeline of a dp x pp grid (rank =
    pipe * pp + stage): key (src, dst) -> group of {src, dst}; activations flow (s, s+1),
    gradients (s+1, s). Collective: every rank must call it, in the same program order."""
    if not dist.is_initialized() or pp < 2:
        return None
    links = {}
    for pipe in range(dp):
        for s in range(pp - 1):
            a, b = pipe * pp + s, pipe * pp + s + 1
            links[(a, b)] = dist.new_group([a, b])
            links[(b, a)] = dist.new_group([a, b])
    return links


def _warm_links(links: dict, me: int, device) -> None:
    """Initialise my link communicators in one global order (a blocking 1-element exchange per
    link), so no lazy communicator rendezvous happens inside the asynchronous schedule."""
    for (src, dst) in sorted(links):
        if me not in (src, dst):
            continue
        g = links[(src, dst)]
        dev = "cpu" if dist.get_backend(g) == "gloo" else device
        t = torch.zeros(1, dtype=torch.float32, device=dev)
        if me == src:
            dist.send(t, dst, group=g)
        else:
            dist.recv(t, src, group=g)


def grid_ranks(rank: int, dp: int, pp: int):
    """2-D DP x PP grid (pipeline-major like the reference: pipeline_id = rank // pp,
    stage = rank % pp; DP groups = same stage across pipelines, e.g. {0,3},{1,4},{2,5})."""
    pipe, stage = divmod(rank, pp)
    pipe_ranks = [pipe * pp + s for s in range(pp)]
    dp_ranks = [p * pp + stage for p in range(dp)]
    return pipe, stage, pipe_ranks, dp_ranks
