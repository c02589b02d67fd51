"""Fused optimizers over a model's flat ParamStore (one kernel for all params of all clients).

Drop-in for the reference's ``torch.optim.SGD`` (hfl_complete.py:196,319), ``Adam`` (intro.py:22,
generative-modeling.py:154) and ``AdamW`` (vfl.py:50): same hyper-parameters and update rules,
but one launch over ``G*P`` floats that also refreshes the bf16 weight shadow.
"""
from __future__ import annotations

import torch

from .ops import functional as Fn


def _store_of(params):
    from .models.net import Net
    from .models.params import ParamStore
    if isinstance(params, Net):
        return params.store
    if isinstance(params, ParamStore):
        return params
    store = getattr(params, "store", None)
    if store is None:
        raise TypeError("ddl25spring_amd optimizers take a native Net / ParamStore "
                        "(use torch.optim for plain torch modules)")
    return store


class _Base:
    def __init__(self, params):
        self.store = _store_of(params)
        self._g = (0, self.store.G)

    def zero_grad(self, set_to_none: bool = False):
        g0, g1 = self._g
        self.store.grad[g0:g1].zero_()

    def select(self, g0: int, g1: int):
        """Restrict the next steps to client slots [g0, g1)."""
        self._g = (g0, g1)
        return self

    def _rows(self, t):
        g0, g1 = self._g
        return t[g0:g1]

    def _shadow_rows(self):
        sh = self.store.shadow16
        return None if sh is None else self._rows(sh)


class SGD(_Base):
    def __init__(self, params, lr: float, momentum: float = 0.0, dampening: float = 0.0,
                 weight_decay: float = 0.0, nesterov: bool = False):
        super().__init__(params)
        self.lr, self.momentum, self.dampening = lr, momentum, dampening
        self.weight_decay, self.nesterov = weight_decay, nesterov
        self.mom = torch.zeros_like(self.store.data) if momentum else None
        self.steps = 0

    def step(self, grad_scale: float = 1.0):
        st = self.store
        Fn.sgd_step(self._rows(st.data), self._rows(st.grad),
                    None if self.mom is None else self._rows(self.mom), self._shadow_rows(),
                    self.lr, self.weight_decay, self.momentum, self.dampening, self.nesterov,
                    first_step=(self.steps == 0), grad_scale=grad_scale)
        st._shadow_version = st.data._version
        self.steps += 1

    def step_direct(self, grad_scale: float = 1.0):
        """Finish a step whose conv-weight part the backward already applied
        (``ParamStore.direct_update``): shadow refresh for those, plain SGD + gradient zeroing for
        the rest, in one launch. Only for momentum- and weight-decay-free SGD, unscaled gradients
        (the WGRAD launches already added the unscaled ``-lr * dW``)."""
        assert self.mom is None and self.weight_decay == 0.0
        if grad_scale != 1.0:
            raise ValueError("step_direct: the direct columns were stepped unscaled inside the backward")
        st = self.store
        Fn.sgd_direct_step(self._rows(st.data), self._rows(st.grad), self._shadow_rows(),
                           st.direct_map, self.lr, grad_scale)
        st._shadow_version = st.data._version
        self.steps += 1

    def reset_state(self):
        self.steps = 0
        if self.mom is not None:
            self.mom.zero_()


class Adam(_Base):
    decoupled = False

    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0):
        super().__init__(params)
        self.lr, self.betas, self.eps, self.weight_decay = lr, betas, eps, weight_decay
        self.m = torch.zeros_like(self.store.data)
        self.v = torch.zeros_like(self.store.data)
        self.t = 0

    def step(self, grad_scale: float = 1.0):
        self.t += 1
        st = self.store
        Fn.adam_step(self._rows(st.data), self._rows(st.grad), self._rows(self.m), self._rows(self.v),
                     self._shadow_rows(), self.lr, self.betas[0], self.betas[1], self.eps,
                     self.weight_decay, self.t, self.decoupled, grad_scale)
        st._shadow_version = st.data._version

    def reset_state(self):
        self.t = 0
        self.m.zero_()
        self.v.zero_()


class AdamW(Adam):
    decoupled = True

    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.01):
        super().__init__(params, lr, betas, eps, weight_decay)


class FlatAdam:
    """Adam / AdamW for plain ``torch.nn.Module`` parameters (the VFL / VAE / LLaMA nets): every
    parameter (and its .grad) is re-pointed into ONE contiguous fp32 buffer, so a step is a single
    fused HIP launch instead of torch's per-tensor foreach chain. Same update rule as
    ``torch.optim.Adam``/``AdamW`` (vfl.py:50, exercise_3.py:190, intro.py:22).

    ``zero_grad`` zeroes in place (grads must stay views of the flat buffer); parameters whose
    ``requires_grad`` is False are left alone.

    ``fused=True``: backward accumulates weight gradients straight into ``p.grad`` (no zero-filled
    temporary, no AccumulateGrad add; ``autograd_ops._grad_sink``). ``bf16_shadow=True``: a bf16
    copy of the weights, refreshed by the Adam kernel itself, is what the MFMA ops read (no cast
    per forward); call ``sync_shadow()`` after changing parameters outside ``step()``.
    """

    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0, decoupled: bool = False, fused: bool = False,
                 bf16_shadow: bool = False):
        self.params = [p for p in params if p.requires_grad]
        if not self.params:
            raise ValueError("FlatAdam got no trainable parameters")
        dev = self.params[0].device
        # every tensor starts on a 256-byte boundary (same alignment class as a fresh allocation,
        # so BLAS picks the same kernels as for unflattened parameters); gaps stay zero
        self.offsets, n = [], 0
        for p in self.params:
            self.offsets.append(n)
            n += (p.numel() + 63) // 64 * 64
        self.data = torch.zeros(n, dtype=torch.float32, device=dev)
        self.grad = torch.zeros(n, dtype=torch.float32, device=dev)
        with torch.no_grad():
            for p, off in zip(self.params, self.offsets):
                k = p.numel()
                self.data[off:off + k].copy_(p.detach().reshape(-1))
                p.data = self.data[off:off + k].view_as(p)
                p.grad = self.grad[off:off + k].view_as(p)
        self.m = torch.zeros_like(self.data)
        self.v = torch.zeros_like(self.data)
        self.lr, self.betas, self.eps, self.weight_decay = lr, betas, eps, weight_decay
        self.decoupled, self.t = decoupled, 0
        # device-side step counter: the update stays exact when captured in a HIP graph
        self.t_dev = torch.zeros(1, dtype=torch.int64, device=dev) if dev.type == "cuda" else None
        self.shadow = None
        if bf16_shadow and dev.type == "cuda":
            self.shadow = torch.empty(n, dtype=torch.bfloat16, device=dev)
            self.sync_shadow()
            for p, off in zip(self.params, self.offsets):
                p._ddl_bf16 = self.shadow[off:off + p.numel()].view_as(p)
        if fused:
            for p in self.params:
                p._ddl_fuse_grad = True

    def sync_shadow(self):
        if self.shadow is not None:
            Fn.to_bf16(self.data, out=self.shadow)

    def zero_grad(self, set_to_none: bool = False):
        self.grad.zero_()
        for p, g in zip(self.params, self._views()):
            if p.grad is None or p.grad.data_ptr() != g.data_ptr():
                p.grad = g  # autograd replaced it (e.g. first backward after set_to_none)

    def _views(self):
        for p, off in zip(self.params, self.offsets):
            yield self.grad[off:off + p.numel()].view_as(p)

    @torch.no_grad()
    def step(self):
        for p, g in zip(self.params, self._views()):
            if p.grad is not None and p.grad.data_ptr() != g.data_ptr():
                # grads live elsewhere (e.g. the DP bucketer's all-reduce buckets): copy, and
                # leave p.grad pointing where the bucketer (and fused backward) accumulate
                g.copy_(p.grad)
        self.t += 1
        if self.t_dev is not None:
            Fn.u64_add(self.t_dev, 1)
        Fn.adam_step(self.data, self.grad, self.m, self.v, self.shadow, self.lr, self.betas[0],
                     self.betas[1], self.eps, self.weight_decay, self.t, self.decoupled,
                     step_dev=self.t_dev)


class SlotAdam:
    """Adam for CLIENT-BATCHED ``nn.Module`` parameters: every parameter is [S, *shape] (slot s =
    one client's copy). Storage is slot-major ``data[S, P]`` (a row = one client's whole model, the
    parameters are strided views of it, rows aligned like ``FlatAdam``'s flat buffer so a row has
    exactly a single-client FlatAdam's layout), and each row has its own device step counter, so
    clients that joined different numbers of rounds keep their own bias correction while ONE fused
    launch steps the first ``rows`` slots (csrc/kernels/optim.hip adam_kernel, row_len > 0).
    Backward accumulates weight gradients straight into the slot rows (``_ddl_fuse_grad``,
    ops/grouped.py). ``bf16_shadow``: a bf16 image of the rows, refreshed by the same launch, is
    what the bf16 MFMA ops read."""

    def __init__(self, params, slots: int, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0, bf16_shadow: bool = False):
        self.params = [p for p in params if p.requires_grad]
        S = self.S = slots
        dev = self.params[0].device
        self.offsets, n = [], 0
        for p in self.params:
            if p.shape[0] != S:
                raise ValueError(f"SlotAdam: parameter of shape {tuple(p.shape)} is not [{S}, ...]")
            self.offsets.append(n)
            n += (p[0].numel() + 63) // 64 * 64
        self.P = n
        self.data = torch.zeros(S, n, dtype=torch.float32, device=dev)
        self.grad = torch.zeros_like(self.data)
        self.m = torch.zeros_like(self.data)
        self.v = torch.zeros_like(self.data)
        self.shadow = torch.empty(S, n, dtype=torch.bfloat16, device=dev) \
            if bf16_shadow and dev.type == "cuda" else None
        with torch.no_grad():
            for p, off in zip(self.params, self.offsets):
                k = p[0].numel()
                self.data[:, off:off + k].copy_(p.detach().reshape(S, k))
                p.data = self.data[:, off:off + k].view(p.shape)
                p.grad = self.grad[:, off:off + k].view(p.shape)
                p._ddl_fuse_grad = True
                if self.shadow is not None:
                    p._ddl_bf16 = self.shadow[:, off:off + k].view(p.shape)
        self.sync_shadow()
        self.lr, self.betas, self.eps, self.weight_decay = lr, betas, eps, weight_decay
        self.t = [0] * S  # host step counts (CPU path; the device path reads t_dev)
        self.t_dev = torch.zeros(S, dtype=torch.int64, device=dev) if dev.type == "cuda" else None

    def sync_shadow(self):
        if self.shadow is not None:
            Fn.to_bf16(self.data, out=self.shadow)

    def zero_grad(self):
        self.grad.zero_()

    @torch.no_grad()
    def step(self, rows: int | None = None):
        r = self.S if rows is None else rows
        for i in range(r):
            self.t[i] += 1
        if self.t_dev is not None:
            self.t_dev[:r].add_(1)
        Fn.adam_step(self.data[:r].reshape(-1), self.grad[:r].reshape(-1), self.m[:r].reshape(-1),
                     self.v[:r].reshape(-1), None if self.shadow is None else self.shadow[:r].reshape(-1),
                     self.lr, self.betas[0], self.betas[1], self.eps, self.weight_decay, self.t[:r], False,
                     step_dev=None if self.t_dev is None else self.t_dev[:r], row_len=self.P)


class FlatAdamW(FlatAdam):
    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.01):
        super().__init__(params, lr, betas, eps, weight_decay, decoupled=True)


def make_adam(params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
              weight_decay: float | None = None, decoupled: bool = False):
    """``torch.optim.Adam``/``AdamW`` semantics (AdamW's default weight_decay 0.01) for plain
    ``nn.Module`` parameters: the fused single-launch ``FlatAdam`` when they live on the GPU,
    ``torch.optim`` on the CPU (where the golden tests pin torch's exact arithmetic)."""
    params = [p for p in params if p.requires_grad]
    wd = (0.01 if decoupled else 0.0) if weight_decay is None else weight_decay
    if params and params[0].is_cuda:
        return FlatAdam(params, lr=lr, betas=betas, eps=eps, weight_decay=wd, decoupled=decoupled)
    cls = torch.optim.AdamW if decoupled else torch.optim.Adam
    return cls(params, lr=lr, betas=betas, eps=eps, weight_decay=wd)
