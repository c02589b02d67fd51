"""Federated DCGAN (FedAvg over generator AND discriminator weights) [NS].

BASELINE config "federated DCGAN on 2xMI355X": each client trains a local (G, D) pair on its
private image shard for ``local_steps`` Adam steps, then the server takes the n_k-weighted average
of both networks (and of the BN running statistics), exactly as FedAvgServer does for classifiers
(reference hfl_complete.py:336-390 is the aggregation template). One rank per GPU; client c
lives on rank c % world for the whole run (its Adam state stays there, like a real device); the
weighted sums of all ranks meet in ONE all-reduce per round over a flat fp32 buffer
(G params | D params | BN buffers).

Precision (``precision``): "fp32" by default — the reference's generative lab trains in fp32
(lab/tutorial_2a/generative-modeling.py:13-130) — every layer on the fp32 kernels; "bf16" runs
bf16 MFMA operands / activations with fp32 master weights.

Batch indices AND generator noise of a client's round are a pure function of that client's
(round, client) seed (Philox, ``Fn.gan_inputs``: generated on the device by one kernel, by its
numpy twin on the CPU), so a client trains on the same data whatever slot or rank it lands on.

Each client keeps its own Adam moments and step count across rounds, as a real client device
would.

Client-batched engine (``batched``, the default on the GPU): all of a rank's clients of the round
train TOGETHER — G and D hold S client slots ([S, ...] slot tensors, models.dcgan.Grouped*), every
layer of every client is ONE grouped launch (ops/grouped.py), one SlotAdam launch steps all slots
with per-client step counters, and the round's ``local_steps`` steps of all slots replay from ONE
HIP graph per slot count. The round's inputs are made on the device from a [G, 3] (seed, n,
offset) descriptor (one small asynchronous upload); the n_k-weighted aggregation is the native
``weighted_sum`` (products rounded, added in slot order) over the flat (G | D | BN) rows; then the
all-reduce. With ``sync_rounds = False`` a round enqueues all of that without any host sync (the
losses stay on the device until ``run`` returns). Adam state stays in its slot while the slot keeps
its client (client_fraction 1: never copied). W ranks reproduce the single-process run up to the
all-reduce's summation order (tests/test_gan_multirank_cpu.py).

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
from ..ops import functional as Fn
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
                 use_graph: bool = True, batched: bool | None = None, precision: str = "fp32"):
        self.ctx = ctx
        self.rank = ctx.rank if ctx else 0
        self.world = ctx.world if ctx else 1
        self.device = torch.device(device) if device is not None else client_data[0].device
        torch.manual_seed(seed)
        self.precision = precision
        self.G = Generator(nz, ngf, precision=precision).to(self.device)
        self.D = Discriminator(ndf, precision=precision).to(self.device)
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
        # False: rounds run without host syncs (no per-round wall time / loss read; run() reads the
        # losses once at the end), as FedAvg's unsynchronised rounds (fl/algorithms.py)
        self.sync_rounds = True
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

    def _client_seed(self, c: int, r: int) -> int:
        # round stride = all clients (not K): no two (round, client) pairs share a stream
        return self.seed + int(c) + 1 + r * len(self.data)

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
            if G not in self._bidx:
                self._bidx[G] = torch.empty(self.local_steps, G * B, dtype=torch.int64, device=self.device)
                self._bz[G] = torch.empty(self.local_steps, G, B, nz, device=self.device)
            # the sequential engine's per-(round, client) streams: same batches, same noise
            desc = [(self._client_seed(c, r), len(self.data[c]), self._off[c]) for c in mine]
            Fn.gan_inputs(desc, self.local_steps, B, nz, self._bidx[G], self._bz[G])
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
            acc = self._aggregate_slots(mine, G, wsum)
        else:
            acc = torch.zeros_like(self._flat())
            ld = lg = None
        if self.ctx and self.world > 1:
            self.ctx.all_reduce(acc)
        self._load_flat(acc)
        self._finish_round(res, t0, ld, lg, G)

    def _aggregate_slots(self, mine, G, wsum):
        """The rank's n_k-weighted partial FedAvg of its G slots in ``_flat``'s layout: on the device
        the native weighted sum (aggregate.hip: products rounded, added in slot order) of the slot
        rows of (G | D | BN buffers); the CPU path the same with torch ops."""
        oG, oD = self.gtr.optG, self.gtr.optD
        cvals = [float(self.n[c] / wsum) for c in mine]
        with torch.no_grad():
            if self.device.type == "cuda" and hasattr(self.optG, "data"):
                coef = torch.tensor(cvals, dtype=torch.float32).pin_memory().to(self.device, non_blocking=True)
                acc = torch.empty(self._flat_numel(), dtype=torch.float32, device=self.device)
                off = 0
                for rows in [oG.data[:G], oD.data[:G]] + [gb[:G].reshape(G, -1) for gb in self._gbufs]:
                    n = rows.shape[1]
                    Fn.weighted_sum(rows, coef, acc[off:off + n])
                    off += n
                return acc
            coef = torch.tensor(cvals, dtype=torch.float32, device=self.device).view(G, 1)
            parts = [self._row_global((coef * oG.data[:G]).sum(0), self.G, oG),
                     self._row_global((coef * oD.data[:G]).sum(0), self.D, oD)]
            parts += [(coef.view(G, *([1] * (gb.dim() - 1))) * gb[:G]).sum(0).reshape(-1) for gb in self._gbufs]
            return torch.cat(parts)

    def _flat_numel(self) -> int:
        """Length of the flat (G | D | BN) buffer of ``_flat``."""
        if not hasattr(self, "_flat_len"):
            self._flat_len = sum(t.numel() for t in self._global_tensors())
        return self._flat_len

    def _finish_round(self, res, t0, ld, lg, nloc):
        """Round bookkeeping. Synchronised rounds: device sync, peer-read barrier check, wall time
        and the losses as floats. Unsynchronised: the losses stay device tensors (``run`` reads them
        once at the end) and the round leaves no host sync behind."""
        div = max(1, nloc)
        if self.sync_rounds or self.device.type != "cuda":
            if self.device.type == "cuda":
                torch.cuda.synchronize()
            if self.ctx is not None:
                self.ctx.check_comm()  # a peer-read all-reduce timeout must not load a corrupt aggregate silently
            res.wall_time.append(time.perf_counter() - t0)
            res.loss_d.append(float(ld) / div if ld is not None else 0.0)
            res.loss_g.append(float(lg) / div if lg is not None else 0.0)
        else:  # (device tensor, divisor): read and divided on the host in _settle, as above
            res.loss_d.append((ld.detach().clone(), div) if ld is not None else 0.0)
            res.loss_g.append((lg.detach().clone(), div) if lg is not None else 0.0)
        res.rounds += 1
        self.round_idx += 1

    # ---------------------------------------------------------------------------------------
    def run(self, rounds: int) -> GANRunResult:
        res = GANRunResult()
        if self.batched:
            for _ in range(rounds):
                self._round_batched(res)
            return self._settle(res)
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
                data = self.data[int(c)]
                if int(c) not in self._idx:
                    self._idx[int(c)] = torch.empty(self.local_steps, self.batch_size, dtype=torch.int64,
                                                    device=data.device)
                    self._z[int(c)] = torch.empty(self.local_steps, self.batch_size, self.G.nz, device=data.device)
                Fn.gan_inputs([(self._client_seed(c, r), len(data), 0)], self.local_steps, self.batch_size,
                              self.G.nz, self._idx[int(c)], self._z[int(c)])
                if self.use_graph:
                    if int(c) not in self._graphs:
                        me = weakref.proxy(self)
                        self._graphs[int(c)] = CapturedStep(lambda c=int(c): me._local_steps(c), warmup=1)
                    ld, lg = self._graphs[int(c)]()
                else:
                    ld, lg = self._local_steps(int(c))
                res.samples += self.batch_size * self.local_steps
                ld_sum = ld_sum + ld.detach()
                lg_sum = lg_sum + lg.detach()
                self._swap_out(int(c))
                acc.add_(self._flat(), alpha=float(self.n[c] / wsum))
            if self.ctx and self.world > 1:
                self.ctx.all_reduce(acc)
            self._load_flat(acc)
            self._finish_round(res, t0, ld_sum if len(mine) else None, lg_sum if len(mine) else None, len(mine))
        return self._settle(res)

    def _settle(self, res):
        """Unsynchronised rounds: one device sync, the comm check and the loss reads, at the end."""
        if any(isinstance(v, tuple) for v in res.loss_d + res.loss_g):
            if self.device.type == "cuda":
                torch.cuda.synchronize()
            if self.ctx is not None:
                self.ctx.check_comm()
            val = lambda v: float(v[0]) / v[1] if isinstance(v, tuple) else v  # noqa: E731
            res.loss_d = [val(v) for v in res.loss_d]
            res.loss_g = [val(v) for v in res.loss_g]
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
