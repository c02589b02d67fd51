"""Flat, client-batched parameter storage.

Every model owns ONE ``ParamStore``: all trainable tensors of all ``G`` co-resident clients live in
a single fp32 buffer ``data[G, P]`` (plus ``grad[G, P]`` and a bf16 ``shadow[G, P]`` read by the
MFMA kernels); non-trainable state (BatchNorm running statistics) lives in ``buffers[G, B]``.

Consequences of this layout (the MI355X-first replacement for the reference's per-client
``nn.Module`` replicas and host round-trips, hfl_complete.py:146-151,323-332,356):
  * the optimizer is one fused kernel over ``G*P`` elements (and refreshes the shadow);
  * FedAvg is one weighted row-reduction + one RCCL all-reduce of ``P`` floats;
  * server -> client download is one broadcast kernel, weights never leave HBM;
  * the buffers are sized per GPU for 288 GB HBM: thousands of MnistCnn / hundreds of
    ResNet-18 clients fit on one device.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field
from typing import Callable

import torch

from ..ops import functional as Fn

# Storage dtype of the weight shadow for CPU stores. bf16 mirrors the device numerics; tests flip
# it (together with ops.reference._bf) to fp32 to check the fwd/bwd *logic* exactly.
CPU_SHADOW_DTYPE = torch.bfloat16

# Compute precision of native nets: "bf16" (bf16 MFMA operands and activations, fp32 master
# weights / accumulation) or "fp32" (the reference's precision, lab/tutorial_1a/hfl_complete.py:
# 39-80: fp32 activations and weights end to end on the exact-fp32 MFMA, conv_f32.hip; the
# kernels read the fp32 master weights directly, there is no shadow). DDL_PRECISION sets the
# default for nets built without an explicit precision.
PRECISIONS = ("bf16", "fp32")
_DEFAULT_PRECISION = [os.environ.get("DDL_PRECISION", "bf16")]


def default_precision() -> str:
    return _DEFAULT_PRECISION[0]


def set_default_precision(p: str) -> None:
    if p not in PRECISIONS:
        raise ValueError(f"precision must be one of {PRECISIONS}, got {p!r}")
    _DEFAULT_PRECISION[0] = p


@dataclass
class Spec:
    name: str
    shape: tuple
    init: Callable[[torch.Tensor, torch.Generator], None]
    buffer: bool = False
    offset: int = 0
    numel: int = 0
    direct: bool = False  # gradient comes only from WGRAD launches (direct-SGD eligible)


def kaiming_uniform_(fan_in: int, a: float = math.sqrt(5)):
    """torch's default nn.Conv2d / nn.Linear weight init (kaiming_uniform_, a=sqrt(5))."""
    gain = math.sqrt(2.0 / (1 + a * a))
    bound = gain * math.sqrt(3.0 / fan_in)

    def f(t, gen):
        t.uniform_(-bound, bound, generator=gen)
    return f


def uniform_bias_(fan_in: int):
    bound = 1.0 / math.sqrt(fan_in) if fan_in > 0 else 0.0

    def f(t, gen):
        t.uniform_(-bound, bound, generator=gen)
    return f


def const_(v: float):
    def f(t, gen):
        t.fill_(v)
    return f


def normal_(std: float, mean: float = 0.0):
    def f(t, gen):
        t.normal_(mean, std, generator=gen)
    return f


class ParamStore:
    def __init__(self, groups: int = 1):
        self.G = groups
        self.specs: dict[str, Spec] = {}
        self.P = 0
        self.B = 0
        self.data = self.grad = self.shadow = self.buffers = None
        self.device = torch.device("cpu")
        self._shadow_version = -1
        self.direct_map = None   # uint8 [P/16]: chunks of direct-SGD-eligible params
        self.n_direct = 0
        self.direct_mode = False
        self._direct_lr = 0.0

    # ---------------------------------------------------------------- declaration
    def add(self, name: str, shape, init, buffer: bool = False, direct: bool = False) -> str:
        if name in self.specs:
            raise KeyError(f"duplicate parameter {name}")
        shape = tuple(int(s) for s in shape)
        n = math.prod(shape)
        # 16-element (64 B) alignment so every view starts on a vector boundary
        if buffer:
            off = self.B
            self.B += (n + 15) // 16 * 16
        else:
            off = self.P
            self.P += (n + 15) // 16 * 16
        self.specs[name] = Spec(name, shape, init, buffer, off, n, direct and not buffer)
        return name

    def param_layout(self) -> list:
        """[[name, offset, numel], ...] of the trainable params in the flat ``data`` row."""
        return [[n, s.offset, s.numel] for n, s in self.specs.items() if not s.buffer]

    def remap_flat(self, flat: torch.Tensor, layout: list) -> torch.Tensor:
        """A flat parameter row written with ``layout`` ([[name, offset, numel], ...]) in this
        store's layout (by name)."""
        out = torch.zeros(max(self.P, 16), dtype=flat.dtype, device=flat.device)
        for name, off, n in layout:
            s = self.specs[name]
            assert s.numel == n and not s.buffer, name
            out[s.offset:s.offset + n] = flat[off:off + n]
        return out

    def _direct_map(self):
        """uint8 [P/16]: 1 on the 16-column chunks of direct-eligible params (every spec starts on
        a 16-element boundary and pads to one), read by the direct-SGD finishing launch."""
        m = torch.zeros(max(self.P, 16) // 16, dtype=torch.uint8)
        for s in self.specs.values():
            if s.direct and not s.buffer:
                m[s.offset // 16:(s.offset + s.numel + 15) // 16] = 1
        self.n_direct = int(m.sum()) * 16
        return m

    # ---------------------------------------------------------------- materialise
    def materialize(self, device, seed: int = 0, generator: torch.Generator | None = None,
                    fp32: bool = False):
        """fp32=True: the kernels read the fp32 master weights themselves (``shadow`` IS ``data``)."""
        device = torch.device(device)
        self.device = device
        G = self.G
        gen = generator if generator is not None else torch.Generator().manual_seed(seed)
        data = torch.zeros(G, max(self.P, 16), dtype=torch.float32)
        bufs = torch.zeros(G, max(self.B, 16), dtype=torch.float32)
        # identical init for every client slot (FedAvg clients start from the server model)
        for s in self.specs.values():
            t = torch.empty(s.shape, dtype=torch.float32)
            s.init(t, gen)
            tgt = bufs if s.buffer else data
            tgt[:, s.offset:s.offset + s.numel] = t.reshape(1, -1)
        self.data = data.to(device)
        self.direct_map = self._direct_map().to(device)
        self.buffers = bufs.to(device)
        self.grad = torch.zeros_like(self.data)
        if fp32:
            self.shadow = self.data
        else:
            sdt = torch.bfloat16 if device.type != "cpu" else CPU_SHADOW_DTYPE
            self.shadow = torch.empty(self.data.shape, dtype=sdt, device=device)
        self.sync_shadow()
        return self

    @property
    def shadow16(self):
        """The separate bf16 weight shadow the optimizers refresh, or None when the kernels read
        the fp32 master weights (fp32 precision)."""
        return None if self.shadow is self.data else self.shadow

    def sync_shadow(self):
        if self.shadow is self.data:
            pass
        elif self.shadow.dtype == torch.float32:
            self.shadow.copy_(self.data)
        else:
            Fn.to_bf16(self.data, self.shadow)
        self._shadow_version = self.data._version

    def ensure_shadow(self):
        """Re-cast the bf16 shadow if the fp32 master was modified outside our fused optimizers."""
        if self.data._version != self._shadow_version:
            self.sync_shadow()

    # ---------------------------------------------------------------- views
    _gsl = slice(None)

    def _view(self, flat: torch.Tensor, s: Spec) -> torch.Tensor:
        return flat[self._gsl, s.offset:s.offset + s.numel].unflatten(1, s.shape)

    class _Select:
        def __init__(self, store, g0, g1):
            self.store, self.sl = store, slice(g0, g1)

        def __enter__(self):
            self.prev = self.store._gsl
            self.store._gsl = self.sl
            return self.store

        def __exit__(self, *a):
            self.store._gsl = self.prev

    def select(self, g0: int, g1: int):
        """Context: layer views cover only client slots [g0, g1) (ragged tail steps)."""
        return ParamStore._Select(self, g0, g1)

    def param(self, name):
        return self._view(self.data, self.specs[name])

    def grad_of(self, name):
        s = self.specs[name]
        if self.direct_mode and s.direct:
            v = self._view(self.data, s)
            v._ddl_wscale = -self._direct_lr  # read by Fn.wgrad_scale: the WGRAD adds -lr * dW
            return v
        return self._view(self.grad, s)

    class _Direct:
        def __init__(self, store, lr):
            self.store, self.lr = store, float(lr)

        def __enter__(self):
            st = self.store
            self.prev = (st.direct_mode, st._direct_lr)
            st.direct_mode, st._direct_lr = True, self.lr
            return st

        def __exit__(self, *a):
            self.store.direct_mode, self.store._direct_lr = self.prev

    def direct_update(self, lr: float):
        """Context: the conv weights' (``Spec.direct``) WGRAD launches add ``-lr * dW`` straight into
        the fp32 master weights instead of a zeroed gradient buffer — a plain SGD step (no momentum /
        weight decay) fused into the backward. Finish the step with ``optim.SGD.step_direct``."""
        return ParamStore._Direct(self, lr)

    def shadow_of(self, name):
        return self._view(self.shadow, self.specs[name])

    def buffer(self, name):
        return self._view(self.buffers, self.specs[name])

    def zero_grad(self):
        self.grad.zero_()

    def param_names(self):
        return [n for n, s in self.specs.items() if not s.buffer]

    def buffer_names(self):
        return [n for n, s in self.specs.items() if s.buffer]

    def num_params(self, true_shapes: bool = True) -> int:
        return sum(s.numel for s in self.specs.values() if not s.buffer)

    # ---------------------------------------------------------------- (de)serialisation
    def state_dict(self, group: int = 0) -> dict[str, torch.Tensor]:
        out = {}
        for n, s in self.specs.items():
            src = self.buffers if s.buffer else self.data
            out[n] = src[group, s.offset:s.offset + s.numel].reshape(s.shape).detach().cpu().clone()
        return out

    def load_state_dict(self, sd: dict[str, torch.Tensor], group: int | None = None):
        groups = range(self.G) if group is None else [group]
        with torch.no_grad():
            for n, t in sd.items():
                s = self.specs[n]
                dst = self.buffers if s.buffer else self.data
                for g in groups:
                    dst[g, s.offset:s.offset + s.numel] = t.reshape(-1).to(dst.device, torch.float32)
        self.sync_shadow()

    def copy_group(self, src_group: int, dst_groups=None):
        dst_groups = range(self.G) if dst_groups is None else dst_groups
        with torch.no_grad():
            for g in dst_groups:
                if g != src_group:
                    self.data[g].copy_(self.data[src_group])
                    self.buffers[g].copy_(self.buffers[src_group])
        self.sync_shadow()
