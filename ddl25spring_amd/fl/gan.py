"""Federated DCGAN (FedAvg over generator AND discriminator weights) [NS].

BASELINE config "federated DCGAN on 2xMI355X": each client trains a local (G, D) pair on its
private image shard for ``local_steps`` Adam steps, then the server takes the n_k-weighted average
of both networks (and of the BN running statistics), exactly as FedAvgServer does for classifiers
(reference hfl_complete.py:336-390 is the aggregation template). One rank per GPU; client c
lives on rank c % world for the whole run (its Adam state stays there, like a real device); the
weighted sums of all ranks meet in ONE all-reduce per round over a flat fp32 buffer
(G params | D params | BN buffers). Batch indices AND generator noise of a client's round are
drawn from that client's own seeded generator, so the result does not depend on how many ranks
share the clients: W ranks reproduce the single-process run.

Each client keeps its own Adam moments and step count across rounds, as a real client device
would.

Client-batched engine (``batched``, the default on the GPU): all of a rank's clients of the round
train TOGETHER — G and D hold S client slots ([S, ...] slot tensors, models.dcgan.Grouped*), every
layer of every client is ONE grouped launch (ops/grouped.py), one SlotAdam launch steps all slots
with per-client step counters, and the round's ``local_steps`` steps of all slots replay from ONE
HIP graph per slot count. Batch indices / noise are drawn per client from the same seeded
generators as the sequential engine (so both engines train the same clients on the same data),
uploaded once per round; download, weighted aggregation and the all-reduce stay on the device over
the flat (G | D | BN) buffers, with one host sync per round (wall time and the loss log). Adam state
stays in its slot while the slot keeps its client (client_fraction 1: never copied).

Sequential engine (``batched=False``; the CPU default): one client after another through a single
(G, D) pair, its Adam state swapped in and out of the fused FlatAdam buffers; on the GPU each
client's steps replay from one HIP graph per client.
"""
from __future__ import annotations

import math
import time
import warnings
import weakref
from dataclasses import dataclass, field

import numpy as np
import torch

from ..models.dcgan import (Discriminator, GANTrainer, Generator, GroupedDiscriminator, GroupedGANTrainer,
                            GroupedGenerator)
from ..runtime.graphs import CapturedStep

# the slot tensors' gradients are strided rows of SlotAdam's [S, P] buffer (CPU autograd path)
warnings.filterwarnings("ignore", message="grad and param do not obey the gradient layout contract")


@dataclass
class GANRunResult:
    rounds: int = 0
    loss_d: list = field(default_factory=list)
    loss_g: list = field(default_factory=list)
    wall_time: list = field(default_factory=list)
    samples: int = 0

    def rounds_per_sec(self):
        return len(self.wall_time) / max(sum(self.wall_time), 1e-9)


def _flat_buffers(mods):
    return [b for m in mods for b in m.buffers() if b.dtype.is_floating_point]


def _row_params(row, mod, slot_opt):
    """Inverse of _param_row: the parameters of a SlotAdam row, concatenated without gaps."""
    return torch.cat([row[off:off + p.numel()] for p, off in
                      zip([p for p in mod.parameters() if p.requires_grad], slot_opt.offsets)])


def _param_row(mod, slot_opt):
    """A single module's parameters in a SlotAdam row layout (CPU torch.optim path)."""
    row = torch.zeros(slot_opt.P, dtype=torch.float32, device=slot_opt.data.device)
    for p, off in zip([p for p in mod.parameters() if p.requires_grad], slot_opt.offsets):
        row[off:off + p.numel()] = p.detach().reshape(-1)
    return row


class FederatedGAN:
    def __init__(self, client_data: list[torch.Tensor], ctx=None, nz: int = 100, ngf: int = 64,
                 ndf: int = 64, lr: float = 2e-4, betas=(0.5, 0.999), local_steps: int = 10,
                 batch_size: int = 64, client_fraction: float = 1.0, seed: int = 0, device=None,
                 use_graph: bool = True, batched: bool | None = None):
        self.ctx = ctx
        self.rank = ctx.rank if ctx else 0
        self.world = ctx.world if ctx else 1
        self.device = torch.device(device) if device is not None else client_data[0].device
        torch.manual_seed(seed)
        self.G = Generator(nz, ngf).to(self.device)
        self.D = Discriminator(ndf).to(self.device)
        self.trainer = GANTrainer(self.G, self.D, lr, betas)
        self.optG, self.optD = self.trainer.optG, self.trainer.optD
        if ctx and self.world > 1:
            for t in self._global_tensors():
                ctx.broadcast(t, 0)
        self.data = client_data
        self.n = np.array([len(d) for d in client_data], dtype=np.float64)
        self.K = max(1, round(client_fraction * len(client_data)))
        self.rng = np.random.default_rng(seed)
        self.local_steps, self.batch_size, self.seed = local_steps, batch_size, seed
        self._state = {}  # client -> (mG, vG, tG, mD, vD, tD, tG_dev, tD_dev)
        self.use_graph = use_graph and self.device.type == "cuda"
        self._idx: dict = {}    # client -> static [local_steps, batch] device index buffer
        self._z: dict = {}      # client -> static [local_steps, batch, nz] generator noise buffer
        self._graphs: dict = {}  # client -> CapturedStep over its local steps
        self.round_idx = 0       # rounds done (seeds the per-round client generators)
        self.batched = (self.device.type == "cuda") if batched is None else bool(batched)
        if self.batched:
            self._init_batched(lr, betas)

    # ---------------------------------------------------------------------------------------
    def _global_tensors(self):
        """Everything FedAvg averages: parameters (the FlatAdam flat buffers on device) + BN stats."""
        if hasattr(self.optG, "data"):
            params = [self.optG.data, self.optD.data]
        else:
            params = [p.data for p in list(self.G.parameters()) + list(self.D.parameters())]
        return params + _flat_buffers([self.G, self.D])

    def _flat(self):
        return torch.cat([t.detach().reshape(-1).float() for t in self._global_tensors()])

    def _load_flat(self, flat):
        off = 0
        with torch.no_grad():
            for t in self._global_tensors():
                k = t.numel()
                t.copy_(flat[off:off + k].view_as(t))
                off += k

    def _swap_in(self, c):
        st = self._state.get(c)
        for opt, i in ((self.optG, 0), (self.optD, 3)):
            if not hasattr(opt, "m"):  # torch.optim.Adam (CPU): per-client state dicts
                if st is None:
                    opt.state.clear()
                else:
                    opt.load_state_dict(st[i])
                continue
            if st is None:
                opt.m.zero_(); opt.v.zero_(); opt.t = 0
                if opt.t_dev is not None:
                    opt.t_dev.zero_()
            else:
                opt.m.copy_(st[i]); opt.v.copy_(st[i + 1]); opt.t = st[i + 2]
                if opt.t_dev is not None:  # the device step counter drives the bias correction
                    opt.t_dev.copy_(st[6 + i // 3])

    def _swap_out(self, c):
        if not hasattr(self.optG, "m"):
            import copy
            self._state[c] = (copy.deepcopy(self.optG.state_dict()), None, None,
                              copy.deepcopy(self.optD.state_dict()), None, None)
        else:
            tdev = [None if o.t_dev is None else o.t_dev.clone() for o in (self.optG, self.optD)]
            self._state[c] = (self.optG.m.clone(), self.optG.v.clone(), self.optG.t,
                              self.optD.m.clone(), self.optD.v.clone(), self.optD.t, *tdev)

    def _local_steps(self, c):
        data, idx, z = self.data[c], self._idx[c], self._z[c]
        ld = lg = None
        for i in range(self.local_steps):
            ld, lg = self.trainer.step(data.index_select(0, idx[i]), z=z[i])
        return ld, lg

    # ------------------------------------------------------------------ client-batched engine
    def _init_batched(self, lr, betas):
        S = self.S = math.ceil(self.K / self.world)
        self.gG = GroupedGenerator(self.G, S).to(self.device)
        self.gD = GroupedDiscriminator(self.D, S).to(self.device)
        self.gtr = GroupedGANTrainer(self.gG, self.gD, S, lr, tuple(betas))
        # this rank's clients (client c lives on rank c % world) in one device tensor: a slot's batch
        # is a row gather with the client's offset folded into the uploaded indices
        self._mine_all = [c for c in range(len(self.data)) if c % self.world == self.rank]
        self._off = {}
        off = 0
        for c in self._mine_all:
            self._off[c] = off
            off += len(self.data[c])
        self._cat = torch.cat([self.data[c] for c in self._mine_all]) if self._mine_all else None
        self._slot_clients = [None] * S
        self._bidx: dict = {}
        self._bz: dict = {}
        self._bgraphs: dict = {}
        self._gbufs = _flat_buffers([self.gG, self.gD])
        self._bufs = _flat_buffers([self.G, self.D])

    def _row_global(self, row, mod, slot_opt):
        """A slot-row vector in ``_flat``'s layout: the FlatAdam buffer itself on the device (same
        aligned layout), the gap-free parameter concatenation with torch.optim on the CPU."""
        opt = self.optG if mod is self.G else self.optD
        return row if hasattr(opt, "data") else _row_params(row, mod, slot_opt)

    def _slot_state_out(self, i):
        """Slot i's Adam state -> its client's entry of ``_state`` (the sequential engine's format)."""
        c = self._slot_clients[i]
        if c is None:
            return
        oG, oD = self.gtr.optG, self.gtr.optD
        tdev = [None if o.t_dev is None else o.t_dev[i:i + 1].clone() for o in (oG, oD)]
        self._state[c] = (oG.m[i].clone(), oG.v[i].clone(), oG.t[i], oD.m[i].clone(), oD.v[i].clone(), oD.t[i],
                          *tdev)

    def _assign_slots(self, mine):
        """Slot order for this round's clients: a client already resident in one of the first
        len(mine) slots stays there (its Adam state is not copied); the others fill the free ones.
        Every displaced slot's state is written back BEFORE any slot loads (a client may move)."""
        G = len(mine)
        order = [None] * G
        rest = []
        for c in mine:
            i = self._slot_clients.index(c) if c in self._slot_clients else -1
            if 0 <= i < G:
                order[i] = c
            else:
                rest.append(c)
        free = [i for i in range(G) if order[i] is None]
        for i, c in zip(free, rest):
            order[i] = c
        for i in range(self.S):
            cur = self._slot_clients[i]
            if cur is not None and (i >= G or order[i] != cur):
                self._slot_state_out(i)
                self._slot_clients[i] = None
        for i, c in enumerate(order):
            self._slot_state_in(i, c)
        return order

    def _slot_state_in(self, i, c):
        if self._slot_clients[i] == c:
            return  # the slot still holds this client's state
        st = self._state.get(c)
        for o, j in ((self.gtr.optG, 0), (self.gtr.optD, 3)):
            if st is None:
                o.m[i].zero_(); o.v[i].zero_(); o.t[i] = 0
                if o.t_dev is not None:
                    o.t_dev[i].zero_()
            else:
                o.m[i].copy_(st[j]); o.v[i].copy_(st[j + 1]); o.t[i] = st[j + 2]
                if o.t_dev is not None:
                    o.t_dev[i:i + 1].copy_(st[6 + j // 3])
        self._slot_clients[i] = c

    def flush_slots(self):
        """Write every slot's Adam state back to ``_state`` (checkpointing)."""
        if not self.batched:
            return
        for i in range(self.S):
            self._slot_state_out(i)
        for o, j in ((self.gtr.optG, 2), (self.gtr.optD, 5)):
            if o.t_dev is not None:  # graph replays advance only the device counters
                for c, st in list(self._state.items()):
                    if st[6 + j // 3] is not None:
                        self._state[c] = tuple(int(st[6 + j // 3].item()) if k == j else v for k, v in enumerate(st))

    def _batched_local(self, G):
        idx, z = self._bidx[G], self._bz[G]
        B = self.batch_size
        ld = lg = None
        for i in range(self.local_steps):
            real = self._cat.index_select(0, idx[i]).view(G, B, *self._cat.shape[1:])
            ld, lg = self.gtr.step(real, z[i])
        return ld, lg

    def _round_batched(self, res):
        r = self.round_idx
        t0 = time.perf_counter()
        chosen = self.rng.choice(len(self.data), self.K, replace=False)
        mine = [int(c) for c in chosen if c % self.world == self.rank]
        G = len(mine)
        wsum = self.n[chosen].sum()
        oG, oD = self.gtr.optG, self.gtr.optD
        if G:
            with torch.no_grad():  # download the global model into the slots in use
                oG.data[:G].copy_(self.optG.data if hasattr(self.optG, "data") else _param_row(self.G, oG))
                oD.data[:G].copy_(self.optD.data if hasattr(self.optD, "data") else _param_row(self.D, oD))
                for gb, b in zip(self._gbufs, self._bufs):
                    gb[:G].copy_(b)
            oG.sync_shadow()
            oD.sync_shadow()
            mine = self._assign_slots(mine)
            B, nz = self.batch_size, self.G.nz
            idx = torch.empty(self.local_steps, G * B, dtype=torch.int64)
            z = torch.empty(self.local_steps, G, B, nz)
            for i, c in enumerate(mine):
                # the sequential engine's per-(round, client) stream: same batches, same noise
                g = torch.Generator(device="cpu").manual_seed(self.seed + c + 1 + r * len(self.data))
                n_c = len(self.data[c])
                idx[:, i * B:(i + 1) * B] = torch.stack([torch.randint(0, n_c, (B,), generator=g)
                                                         for _ in range(self.local_steps)]) + self._off[c]
                z[:, i] = torch.randn(self.local_steps, B, nz, generator=g)
            if G not in self._bidx:
                self._bidx[G] = torch.empty_like(idx, device=self.device)
                self._bz[G] = torch.empty_like(z, device=self.device)
            self._bidx[G].copy_(idx, non_blocking=False)
            self._bz[G].copy_(z, non_blocking=False)
            if self.use_graph:
                if G not in self._bgraphs:
                    # a weak self: no engine <-> graph cycle, so the graph dies with the engine
                    # (refcount), not in a later cyclic GC pass
                    me = weakref.proxy(self)
                    self._bgraphs[G] = CapturedStep(lambda G=G: me._batched_local(G), warmup=1)
                ld, lg = self._bgraphs[G]()
            else:
                ld, lg = self._batched_local(G)
            res.samples += self.batch_size * self.local_steps * G
            coef = torch.tensor(self.n[mine] / wsum, dtype=torch.float32, device=self.device).view(G, 1)
            with torch.no_grad():
                parts = [self._row_global((coef * oG.data[:G]).sum(0), self.G, oG),
                         self._row_global((coef * oD.data[:G]).sum(0), self.D, oD)]
                parts += [(coef.view(G, *([1] * (gb.dim() - 1))) * gb[:G]).sum(0).reshape(-1) for gb in self._gbufs]
                acc = torch.cat(parts)
        else:
            acc = torch.zeros_like(self._flat())
            ld = lg = None
        if self.ctx and self.world > 1:
            self.ctx.all_reduce(acc)
        self._load_flat(acc)
        if self.device.type == "cuda":
            torch.cuda.synchronize()
        res.wall_time.append(time.perf_counter() - t0)
        # the grouped losses are sums over the slots' own mean losses: / G = the clients' mean
        res.loss_d.append(float(ld) / G if G else 0.0)
        res.loss_g.append(float(lg) / G if G else 0.0)
        res.rounds += 1
        self.round_idx += 1

    # ---------------------------------------------------------------------------------------
    def run(self, rounds: int) -> GANRunResult:
        res = GANRunResult()
        if self.batched:
            for _ in range(rounds):
                self._round_batched(res)
            return res
        for _ in range(rounds):
            r = self.round_idx
            t0 = time.perf_counter()
            chosen = self.rng.choice(len(self.data), self.K, replace=False)
            mine = [c for c in chosen if c % self.world == self.rank]
            glob = self._flat()
            acc = torch.zeros_like(glob)
            wsum = self.n[chosen].sum()
            ld_sum = lg_sum = 0.0
            for c in mine:
                self._load_flat(glob)
                self._swap_in(int(c))
                # round stride = all clients (not K): no two (round, client) pairs share a stream
                g = torch.Generator(device="cpu").manual_seed(self.seed + int(c) + 1 + r * len(self.data))
                data = self.data[int(c)]
                idx = torch.stack([torch.randint(0, len(data), (self.batch_size,), generator=g)
                                   for _ in range(self.local_steps)])
                z = torch.randn(self.local_steps, self.batch_size, self.G.nz, generator=g)
                if int(c) not in self._idx:
                    self._idx[int(c)] = torch.empty_like(idx, device=data.device)
                    self._z[int(c)] = torch.empty_like(z, device=data.device)
                self._idx[int(c)].copy_(idx)
                self._z[int(c)].copy_(z)
                if self.use_graph:
                    if int(c) not in self._graphs:
                        me = weakref.proxy(self)
                        self._graphs[int(c)] = CapturedStep(lambda c=int(c): me._local_steps(c), warmup=1)
                    ld, lg = self._graphs[int(c)]()
                else:
                    ld, lg = self._local_steps(int(c))
                res.samples += self.batch_size * self.local_steps
                ld_sum += float(ld); lg_sum += float(lg)
                self._swap_out(int(c))
                acc.add_(self._flat(), alpha=float(self.n[c] / wsum))
            if self.ctx and self.world > 1:
                self.ctx.all_reduce(acc)
            self._load_flat(acc)
            if self.device.type == "cuda":
                torch.cuda.synchronize()
            res.wall_time.append(time.perf_counter() - t0)
            res.loss_d.append(ld_sum / max(1, len(mine)))
            res.loss_g.append(lg_sum / max(1, len(mine)))
            res.rounds += 1
            self.round_idx += 1
        return res

    # --------------------------------------------------------------------------- checkpointing
    def state_dict(self) -> dict:
        """This rank's shard: the global (G | D | BN) weights and the sampling stream (identical on
        every rank), and the Adam state of the clients that live on this rank."""
        self.flush_slots()
        clients = {}
        for c, st in self._state.items():
            if self.batched or hasattr(self.optG, "m"):
                clients[int(c)] = {"mG": st[0], "vG": st[1], "tG": st[2], "mD": st[3], "vD": st[4],
                                   "tD": st[5]}
            else:
                clients[int(c)] = {"G": st[0], "D": st[3]}
        return {"flat": self._flat(), "round": self.round_idx,
                "rng": self.rng.bit_generator.state, "clients": clients}

    def load_state_dict(self, sd: dict) -> None:
        self._load_flat(sd["flat"].to(self.device))
        self.round_idx = int(sd["round"])
        self.rng.bit_generator.state = sd["rng"]
        self._state = {}
        if self.batched:
            self._slot_clients = [None] * self.S  # slots reload their clients from _state
        for c, st in sd["clients"].items():
            if "G" in st:
                self._state[int(c)] = (st["G"], None, None, st["D"], None, None)
                continue
            dev = self.device
            opts = (self.gtr.optG, self.gtr.optD) if self.batched else (self.optG, self.optD)
            tdev = [torch.tensor([t], dtype=torch.int64, device=dev) if getattr(o, "t_dev", None) is not None
                    else None for t, o in zip((st["tG"], st["tD"]), opts)]
            self._state[int(c)] = (st["mG"].to(dev), st["vG"].to(dev), int(st["tG"]),
                                   st["mD"].to(dev), st["vD"].to(dev), int(st["tD"]), *tdev)
