"""Distributed vertical FL: split-NN and VFL-VAE across ranks (one party per rank).

The reference runs every party inside one process (lab/tutorial_2b/vfl.py:43-102,
exercise_3.py:113-140); here each feature-holding party is its own rank (one GPU each) and the
label/VAE server is rank ``server`` (default 0). Per mini-batch only cut-layer tensors move, over
RCCL point-to-point on xGMI (gloo on CPU):

  split-NN   party -> server : bottom activations  [B, out_i]
             server -> party : d loss / d activation [B, out_i]
  VFL-VAE    party -> server : client latent       [B, L]
             server -> party : reconstructed latent slice [B, L]
             party -> server : d client-loss / d slice, client loss
             server -> party : d total-loss / d latent (VAE input AND latent-MSE target paths)

Every exchange is one ``batch_isend_irecv`` so all parties move concurrently (no per-party
serialisation, no deadlock by construction). With equal initial weights and batches the result is
identical to the single-process ``VFLNetwork`` / ``VFLVAE`` (tests/test_vfl_cpu.py).
"""
from __future__ import annotations

import torch
import torch.distributed as dist
import torch.nn as nn

from ..ops import tabular_ops as TO
from ..optim import make_adam


def _exchange(sends, recvs, group=None):
    if not (sends or recvs):
        return
    staged = dist.get_backend(group) == "gloo" and any(t.is_cuda for t, _ in sends + recvs)
    if staged:
        # gloo P2P moves host memory only (ranks sharing one GPU): stage through the host
        sends = [(t.cpu(), p) for t, p in sends]
        dev_recvs, recvs = recvs, [(torch.empty(t.shape, dtype=t.dtype), p) for t, p in recvs]
    ops = [dist.P2POp(dist.isend, t, peer, group) for t, peer in sends]
    ops += [dist.P2POp(dist.irecv, t, peer, group) for t, peer in recvs]
    for w in dist.batch_isend_irecv(ops):
        w.wait()
    if staged:
        for (d, _), (h, _) in zip(dev_recvs, recvs):
            d.copy_(h)


def _batches(n, bs):
    nb = (n + bs - 1) // bs
    return [slice(b * bs, (b + 1) * bs) for b in range(nb)]


class SplitNNParty:
    """A feature-holding party: bottom model + its optimizer, features for its columns."""

    def __init__(self, bottom: nn.Module, out_dim: int, server: int = 0, optimizer=None, group=None):
        self.bottom, self.out_dim, self.server, self.group = bottom, out_dim, server, group
        self.opt = optimizer or make_adam(bottom.parameters(), decoupled=True)

    def train_step(self, x):
        self.opt.zero_grad()
        self.bottom.train()
        act = self.bottom(x)
        grad = torch.empty_like(act)
        _exchange([(act.detach().contiguous(), self.server)], [], self.group)
        _exchange([], [(grad, self.server)], self.group)
        act.backward(grad)
        self.opt.step()

    @torch.no_grad()
    def infer(self, x, eval_mode: bool = True):
        self.bottom.train(not eval_mode)
        _exchange([(self.bottom(x).contiguous(), self.server)], [], self.group)

    def fit(self, x, epochs, batch_size, start_epoch: int = 0, on_epoch=None):
        for e in range(start_epoch, epochs):
            for sl in _batches(len(x), batch_size):
                self.train_step(x[sl])
            if on_epoch is not None:
                on_epoch(e + 1)

    def modules(self):
        return {"bottom": self.bottom}


class SplitNNServer:
    """The label holder: top model over the concatenated party activations. With ``local_bottom``
    it is also the *active party* (holds a feature block itself, activation first in the concat),
    so a 2-party split fits on 2 GPUs."""

    def __init__(self, top: nn.Module, parties: list[int], out_dims: list[int], optimizer=None,
                 criterion=None, group=None, local_bottom: nn.Module | None = None):
        self.top, self.parties, self.out_dims, self.group = top, parties, out_dims, group
        self.local = local_bottom
        params = list(top.parameters()) + (list(local_bottom.parameters()) if local_bottom else [])
        self.opt = optimizer or make_adam(params, decoupled=True)
        self.criterion = criterion or nn.CrossEntropyLoss()

    def _recv(self, b, like):
        acts = [torch.empty(b, d, dtype=like.dtype, device=like.device) for d in self.out_dims]
        _exchange([], list(zip(acts, self.parties)), self.group)
        return acts

    def train_step(self, y, x_local=None):
        self.opt.zero_grad()
        self.top.train()
        acts = [a.requires_grad_(True) for a in self._recv(len(y), y)]
        if self.local is not None:
            self.local.train()
            out = self.top([self.local(x_local)] + acts)
        else:
            out = self.top(acts)
        loss = self.criterion(out, y)
        loss.backward()
        self.opt.step()
        # grads go back after the server step: the parties only need them for their own update
        _exchange([(a.grad.contiguous(), p) for a, p in zip(acts, self.parties)], [], self.group)
        lab = y.argmax(1) if y.dim() == 2 else y
        # device scalars: the host never waits on a mini-batch (fit reads them once at the end)
        return loss.detach(), (out.argmax(1) == lab).sum()

    @torch.no_grad()
    def infer(self, n, like, eval_mode: bool = True, x_local=None):
        self.top.train(not eval_mode)
        acts = self._recv(n, like)
        if self.local is not None:
            self.local.train(not eval_mode)
            acts = [self.local(x_local)] + acts
        return self.top(acts)

    def modules(self):
        mods = {"top": self.top}
        if self.local is not None:
            mods["local"] = self.local
        return mods

    def fit(self, y, epochs, batch_size, log=None, x_local=None, start_epoch: int = 0, on_epoch=None):
        """Epochs ``start_epoch`` .. ``epochs``-1; ``on_epoch(e)`` after each (checkpoint hook;
        it sees the history so far as ``self.history``). Returns that history as floats."""
        hist = []
        self.history = hist
        for e in range(start_epoch, epochs):
            tot = torch.zeros((), device=y.device)
            cor = torch.zeros((), dtype=torch.int64, device=y.device)
            bl = _batches(len(y), batch_size)
            for sl in bl:
                l, c = self.train_step(y[sl], None if x_local is None else x_local[sl])
                tot += l
                cor += c
            hist.append(torch.stack([tot / len(bl), cor / len(y)]))
            if log:
                log(e, *hist[-1].tolist())
            if on_epoch is not None:
                on_epoch(e + 1)
        return [tuple(h) for h in torch.stack(hist).tolist()] if hist else []


# ------------------------------------------------------------------------------------ VFL-VAE
class VAEParty:
    def __init__(self, encoder, decoder, latent_dim, server: int = 0, optimizer=None, group=None):
        self.enc, self.dec, self.L, self.server, self.group = encoder, decoder, latent_dim, server, group
        params = list(encoder.parameters()) + list(decoder.parameters())
        self.opt = optimizer or make_adam(params, lr=1e-3)
        self.mse = nn.MSELoss(reduction="sum")

    def train_step(self, x):
        self.opt.zero_grad()
        self.enc.train(); self.dec.train()
        lat = self.enc(x)
        rec = torch.empty_like(lat)
        _exchange([(lat.detach().contiguous(), self.server)], [(rec, self.server)], self.group)
        rec.requires_grad_(True)
        closs = self.mse(self.dec(rec), x)
        closs.backward()
        gl = torch.empty_like(lat)
        _exchange([(rec.grad.contiguous(), self.server),
                   (closs.detach().reshape(1).to(lat.dtype), self.server)],
                  [(gl, self.server)], self.group)
        lat.backward(gl)
        self.opt.step()


class VAEServer:
    def __init__(self, vae, parties, latent_dim, optimizer=None, group=None):
        self.vae, self.parties, self.L, self.group = vae, parties, latent_dim, group
        self.opt = optimizer or make_adam(vae.parameters(), lr=1e-3)
        self.mse = nn.MSELoss(reduction="sum")

    def train_step(self, n, like):
        self.opt.zero_grad()
        self.vae.train()
        P, L = len(self.parties), self.L
        lats = [torch.empty(n, L, dtype=like.dtype, device=like.device) for _ in range(P)]
        _exchange([], list(zip(lats, self.parties)), self.group)
        lat = torch.cat(lats, 1).requires_grad_(True)
        recon, mu, logvar = self.vae(lat)
        slices = [recon[:, i * L:(i + 1) * L] for i in range(P)]
        grads = [torch.empty(n, L, dtype=like.dtype, device=like.device) for _ in range(P)]
        closs = [torch.empty(1, dtype=like.dtype, device=like.device) for _ in range(P)]
        _exchange([(s.detach().contiguous(), p) for s, p in zip(slices, self.parties)],
                  [(g, p) for g, p in zip(grads, self.parties)] +
                  [(c, p) for c, p in zip(closs, self.parties)], self.group)
        sloss = TO.mse_kl(recon, lat, mu, logvar)
        surrogate = sloss + (recon * torch.cat(grads, 1)).sum()
        surrogate.backward()
        self.opt.step()
        _exchange([(lat.grad[:, i * L:(i + 1) * L].contiguous(), p) for i, p in enumerate(self.parties)],
                  [], self.group)
        return sloss.detach() + torch.cat(closs).sum()  # device scalar, no host sync
