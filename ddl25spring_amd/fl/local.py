"""Client-batched local training: E epochs of mini-batch SGD for all G client slots of this GPU
in ONE stream of kernel launches (every launch covers all clients through the group dimension).

Replaces the reference's sequential per-client loop (hfl_complete.py:360-373 calls
``WeightClient.update`` client after client, each one an ``nn.Module`` replica fed by a CPU
DataLoader and copied host<->device every round). Here:
  * weights of all clients live in one flat [G, P] buffer, already on the device;
  * the round's batch plan (which sample ids each client sees at each step) is computed once on
    the host (native planner or torch.randperm for DataLoader-identical order) and uploaded once;
  * the round's steady-state steps (gather+normalise -> fwd -> fused CE -> bwd -> fused SGD, once
    per local step) are captured as ONE HIP graph and replayed, so a round costs one graph launch.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from .. import optim
from ..data.split import plan_epoch
from ..runtime.graphs import CAPTURE_MODE


# Direct SGD (default on the GPU for plain SGD): the conv / Linear weights' WGRAD launches add -lr * dW
# straight into the fp32 master weights (ParamStore.direct_update), so a step skips zero-filling
# and re-reading their gradients and its optimizer launch only refreshes their bf16 shadow.
# DDL_DIRECT_SGD=0 keeps gradient buffer + fused SGD launch.
DIRECT_SGD = os.environ.get("DDL_DIRECT_SGD", "1") != "0"
# Instances of each captured round graph, replayed alternately: ROCm's graph launch waits for the
# same executable's previous launch to finish before it submits the ~7,000 kernel nodes, which left
# the GPU idle ~1 ms at every round boundary even with the host rounds ahead (sync_rounds off);
# with two instances (DDL_ROUND_GRAPHS=2) the host can submit round r+1 while round r runs.
ROUND_GRAPHS = max(1, int(os.environ.get("DDL_ROUND_GRAPHS", "1")))
# Longest step sequence in one captured graph. hipGraphLaunch segfaults once a graph holds between
# 76,145 and 76,930 kernel nodes (measured: 485 ResNet-18 steps of 157 nodes run, 490 crash;
# profiles/graph_node_limit_r6.txt); longer rounds replay a graph per chunk. 128 steps = 20,096
# nodes, a 3.8x margin, and larger chunks gain nothing (26.1-26.3k samples/s from 256 to 485).
GRAPH_MAX_STEPS = max(1, int(os.environ.get("DDL_GRAPH_MAX_STEPS", "128")))
# keep the captured hipGraph_t (torch keep_graph=True) so diagnostics can count its nodes
# (scripts/graph_nodes.py); off by default: the instantiated executable is all a replay needs
KEEP_GRAPH = os.environ.get("DDL_GRAPH_KEEP", "0") == "1"


class LocalTrainer:
    def __init__(self, net, data, lr: float, batch_size: int, momentum: float = 0.0,
                 weight_decay: float = 0.0, planner: str = "native", use_graph: bool | None = None,
                 label_transform=None, direct: bool | None = None):
        self.net, self.data = net, data
        self.B = batch_size
        self.opt = optim.SGD(net, lr=lr, momentum=momentum, weight_decay=weight_decay)
        self.planner = planner
        dev = net.device
        self.use_graph = (dev.type == "cuda") if use_graph is None else (use_graph and dev.type == "cuda")
        eligible = momentum == 0.0 and weight_decay == 0.0 and net.store.n_direct > 0 \
            and getattr(net, "grad_hook", None) is None
        self.direct = eligible and (DIRECT_SGD and dev.type == "cuda" if direct is None else direct)
        self.label_transform = label_transform  # callable(y [G,B], g0, g1) -> y (attacks); with a
        # ``graph_key`` attribute it is pure device ops and may be captured in the round graph
        self._graphs: dict = {}
        self._next: dict = {}
        self.last_loss = None
        # double-buffered pinned staging of the round's batch plan: the host->device copy is then
        # truly asynchronous, so with FederatedBase.sync_rounds off the host plans and enqueues
        # round r+1 while the GPU still runs round r
        self._pinned: dict = {}
        self._pin_slot = 0

    # ---------------------------------------------------------------- one step (eager)
    def _step(self, idx, g0: int, g1: int):
        net, st = self.net, self.net.store
        x, y = self.data.batch(idx)
        if self.label_transform is not None:
            y = self.label_transform(y, g0, g1)
        with st.select(g0, g1):
            if self.direct:  # the previous step_direct left the other gradients zeroed
                with st.direct_update(self.opt.lr):
                    loss, _ = net.train_step(x, y)
                self.opt.select(g0, g1).step_direct()
            else:
                st.grad[g0:g1].zero_()
                loss, _ = net.train_step(x, y)
                self.opt.select(g0, g1).step()
        return loss

    # ---------------------------------------------------------------- graph-captured round
    def _graph_run(self, plan_dev: torch.Tensor, nsteps: int, G: int, tail=None):
        """Steps 0 .. nsteps-1 of the round's plan [steps, G, B] (+ the epoch's short last step
        ``tail`` [G, n], when every slot has the same n) as ONE graph replay: the whole sequence
        of local SGD steps is captured once (every step's batch launch reads its own row of a
        static plan buffer), so a round costs one plan copy and one graph launch. Without the tail
        in the graph, the short step (6,250 samples per client at B=100: 62 steps + 50 samples)
        ran eagerly every round, ~130 host-side launches."""
        if hasattr(self.label_transform, "refresh"):  # this round's device-side transform state
            self.label_transform.refresh(plan_dev.device)
        k0 = 0
        while nsteps - k0 > GRAPH_MAX_STEPS:  # full chunks share one graph (plan rows copied in)
            self._replay(plan_dev[k0:k0 + GRAPH_MAX_STEPS], GRAPH_MAX_STEPS, G, None)
            k0 += GRAPH_MAX_STEPS
        self._replay(plan_dev[k0:nsteps], nsteps - k0, G, tail)

    def _replay(self, plan_dev: torch.Tensor, nsteps: int, G: int, tail):
        key = (G, self.B, nsteps, None if tail is None else tail.shape[-1],
               getattr(self.label_transform, "graph_key", None))
        ents = self._graphs.get(key)
        if ents is None:
            n = ROUND_GRAPHS if self.net.device.type == "cuda" else 1
            ents = [self._capture(plan_dev, nsteps, G, tail) for _ in range(n)]
            self._graphs[key] = ents
            self._next[key] = 0
        ent = ents[self._next[key]]
        self._next[key] = (self._next[key] + 1) % len(ents)
        ent["plan"].copy_(plan_dev[:nsteps])
        if tail is not None:
            ent["tail"].copy_(tail)
        ent["graph"].replay()
        self.last_loss = ent["loss"]

    def _capture(self, plan_dev: torch.Tensor, nsteps: int, G: int, tail=None):
        st, opt = self.net.store, self.opt
        # the warm-up steps really train: snapshot and restore so the first graph step is exact
        snap = (st.data[:G].clone(), st.buffers[:G].clone(),
                None if opt.mom is None else opt.mom[:G].clone(), opt.steps,
                [c.clone() for c in self.net.rng_counters()])
        plan = plan_dev[:nsteps].clone()
        tl = None if tail is None else tail.clone()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for i in range(2):
                self._step(plan[i % nsteps], 0, G)
            if tl is not None:  # the short step's shapes (tuned on first eager use)
                self._step(tl, 0, G)
        torch.cuda.current_stream().wait_stream(s)
        # zero-initialised momentum == torch's "buffer = first grad" when dampening == 0, so the
        # frozen first_step=False inside the graph is exact for every step of a round
        assert opt.dampening == 0.0
        graph = torch.cuda.CUDAGraph(keep_graph=KEEP_GRAPH)
        # DDL_GRAPH_PRIO=1: capture on a high-priority stream, so the step's critical path (the
        # main stream) outranks the side-stream weight gradients (Fn.wgrad_overlap) it overlaps
        cap = torch.cuda.Stream(priority=-1) if os.environ.get("DDL_GRAPH_PRIO", "0") == "1" else None
        with torch.cuda.graph(graph, stream=cap, capture_error_mode=CAPTURE_MODE):
            for i in range(nsteps):
                loss = self._step(plan[i], 0, G)
            if tl is not None:
                loss = self._step(tl, 0, G)
        st.data[:G].copy_(snap[0])
        st.buffers[:G].copy_(snap[1])
        if snap[2] is not None:
            opt.mom[:G].copy_(snap[2])
        opt.steps = snap[3]
        for c, saved in zip(self.net.rng_counters(), snap[4]):
            c.copy_(saved)  # warm-up steps advanced the dropout counters: rewind them too
        st.sync_shadow()
        return {"graph": graph, "plan": plan, "tail": tl, "loss": loss}

    # ---------------------------------------------------------------- public
    def run(self, slot_indices: list[np.ndarray], seeds, epochs: int = 1, generators=None) -> int:
        """Train slots [0, len(slot_indices)) for `epochs` local epochs; returns #samples seen."""
        G = len(slot_indices)
        if G == 0:
            return 0
        self.opt.reset_state()
        if self.direct:
            self.net.store.grad[:G].zero_()  # direct steps keep it zero from here on
        sizes = {len(s) for s in slot_indices}
        samples = 0
        for ep in range(epochs):
            if len(sizes) == 1:
                groups = [(0, G, slot_indices)]
            else:  # unequal client sizes: run each slot on its own (group-sliced views)
                groups = [(g, g + 1, [slot_indices[g]]) for g in range(G)]
            for g0, g1, idxs in groups:
                sd = seeds[g0:g1]
                if self.planner == "torch" and generators is not None:
                    plan = self._torch_plan(idxs, generators[g0:g1])
                else:
                    plan = plan_epoch(idxs, self.B, [int(s) + 7919 * ep for s in sd], True, "native")
                samples += self._run_plan(plan, g0, g1)
        return samples

    def _torch_plan(self, idxs, gens):
        """One epoch of ``DataLoader(subset, B, shuffle=True, generator=gen)`` order. Each
        ``iter(loader)`` consumes, in this order: one int64 ``random_`` (the loader's base seed,
        torch/utils/data/dataloader.py ``_BaseDataLoaderIter.__init__``), the epoch's
        ``randperm(n)``, and a trailing ``randperm(n)`` that ``RandomSampler.__iter__`` draws for
        its ``num_samples % n`` tail (empty here, but the draw still advances the generator)."""
        count = len(idxs[0])
        steps = (count + self.B - 1) // self.B
        out = -np.ones((steps, len(idxs), self.B), dtype=np.int32)
        for g, (ci, gen) in enumerate(zip(idxs, gens)):
            torch.empty((), dtype=torch.int64).random_(generator=gen)
            perm = torch.randperm(count, generator=gen).numpy()
            torch.randperm(count, generator=gen)
            seq = np.asarray(ci)[perm]
            for s in range(steps):
                chunk = seq[s * self.B:(s + 1) * self.B]
                out[s, g, :len(chunk)] = chunk
        return out

    def _upload(self, plan: np.ndarray, dev) -> torch.Tensor:
        if dev.type != "cuda":
            return torch.from_numpy(plan).to(dev)
        slots = self._pinned.get(plan.shape)
        if slots is None:
            slots = [[torch.empty(plan.shape, dtype=torch.int32, pin_memory=True), None] for _ in range(2)]
            self._pinned[plan.shape] = slots
        self._pin_slot ^= 1
        buf, ev = slots[self._pin_slot]
        if ev is not None:
            ev.synchronize()  # the copy that last read this buffer (two uploads ago) is done
        buf.numpy()[...] = plan
        out = buf.to(dev, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        slots[self._pin_slot][1] = ev
        return out

    def _run_plan(self, plan: np.ndarray, g0: int, g1: int) -> int:
        dev = self.net.device
        steps = plan.shape[0]
        full = (plan >= 0).all(axis=(1, 2))
        plan_dev = self._upload(np.ascontiguousarray(plan, dtype=np.int32), dev)
        samples = 0
        G = g1 - g0
        s = 0
        if self.use_graph and g0 == 0:
            nfull = int(np.argmin(full)) if not full.all() else steps  # leading full steps
            tail = None
            if nfull and nfull == steps - 1:  # one short last step, the same n in every slot
                cnt = (plan[-1] >= 0).sum(1)
                n = int(cnt[0])
                if n > 0 and cnt.min() == n and cnt.max() == n and (plan[-1, :, :n] >= 0).all():
                    tail = plan_dev[-1, :, :n].contiguous()
            if nfull:
                self._graph_run(plan_dev, nfull, G, tail)
                samples += nfull * G * self.B + (0 if tail is None else G * tail.shape[-1])
                s = nfull + (0 if tail is None else 1)
        for s in range(s, steps):
            if full[s]:
                self.last_loss = self._step(plan_dev[s], g0, g1)
                samples += G * self.B
            else:
                n = int((plan[s, 0] >= 0).sum())
                if (plan[s] >= 0).sum(1).min() == n and (plan[s] >= 0).sum(1).max() == n:
                    self.last_loss = self._step(plan_dev[s, :, :n].contiguous(), g0, g1)
                    samples += G * n
                else:
                    for g in range(G):
                        m = int((plan[s, g] >= 0).sum())
                        if m:
                            self.last_loss = self._step(plan_dev[s, g:g + 1, :m].contiguous(), g0 + g, g0 + g + 1)
                            samples += m
        return samples
