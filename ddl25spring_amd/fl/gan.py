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

Each client keeps its own Adam moments and step count across rounds (swapped in and out of the
fused FlatAdam buffers), as a real client device would. On the GPU a client's ``local_steps``
steps replay from one HIP graph per client (``runtime.graphs.CapturedStep``): the batch indices
of the round are drawn on the host from the client's seeded generator as before and uploaded into
a static buffer the graph reads.
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field

import numpy as np
import torch

from ..models.dcgan import Discriminator, GANTrainer, Generator
from ..runtime.graphs import CapturedStep


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


class FederatedGAN:
    def __init__(self, client_data: list[torch.Tensor], ctx=None, nz: int = 100, ngf: int = 64,
                 ndf: int = 64, lr: float = 2e-4, betas=(0.5, 0.999), local_steps: int = 10,
                 batch_size: int = 64, client_fraction: float = 1.0, seed: int = 0, device=None,
                 use_graph: bool = True):
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

    # ---------------------------------------------------------------------------------------
    def run(self, rounds: int) -> GANRunResult:
        res = GANRunResult()
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
                        self._graphs[int(c)] = CapturedStep(lambda c=int(c): self._local_steps(c), warmup=1)
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
        clients = {}
        for c, st in self._state.items():
            if hasattr(self.optG, "m"):
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
        for c, st in sd["clients"].items():
            if "G" in st:
                self._state[int(c)] = (st["G"], None, None, st["D"], None, None)
                continue
            dev = self.device
            tdev = [torch.tensor([t], dtype=torch.int64, device=dev) if o.t_dev is not None else None
                    for t, o in ((st["tG"], self.optG), (st["tD"], self.optD))]
            self._state[int(c)] = (st["mG"].to(dev), st["vG"].to(dev), int(st["tG"]),
                                   st["mD"].to(dev), st["vD"].to(dev), int(st["tD"]), *tdev)
