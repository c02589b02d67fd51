"""Net: a sequential container of explicit fwd/bwd layers over one flat ParamStore.

* ``forward_train(x)`` / ``backward(dlogits)`` — the native training path used by the FL engine,
  DP trainer and benchmark (no autograd, graph-capturable).
* ``__call__`` — torch-compatible: with grad enabled the whole net is ONE autograd node, so
  reference-style code (``output = model(data); F.nll_loss(output, target).backward()``) works and
  the backward pass still runs our kernels.
* ``train_step(x, labels)`` — forward + fused CE + backward in one call (client-batched).
"""
from __future__ import annotations

import contextlib
import os

import torch

from ..ops import functional as Fn
from ..ops import reference as ref
from ..ops.workspace import Workspace
from .layers import RELU, ConvUnit, Dropout, Layer
from .params import PRECISIONS, ParamStore, default_precision


class Net:
    def __init__(self, layers: list[Layer], groups: int = 1, num_classes: int | None = None,
                 input_spec: dict | None = None, name: str = "net", precision: str | None = None):
        self.layers = layers
        self.G = groups
        self.num_classes = num_classes
        self.precision = precision or default_precision()
        if self.precision not in PRECISIONS:
            raise ValueError(f"precision must be one of {PRECISIONS}, got {self.precision!r}")
        # the activation dtype travels with the input spec, so data loaders emit it
        self.input_spec = dict(input_spec or {}, dtype=self.precision)
        self.name = name
        self.store = ParamStore(groups)
        # direct-SGD eligibility of Linear weights: all but a classifier head after a global
        # average pool, whose weight gradient the fused head kernel (Fn.head_train) writes
        for i, layer in enumerate(layers):
            if isinstance(layer, ConvUnit) and layer.linear:
                head = i == len(layers) - 1 and i > 0 and layers[i - 1].name == "avgpool"
                layer.direct_w = not head
        for i, layer in enumerate(layers):
            layer.declare(self.store, getattr(layer, "pname", f"{i}.{layer.name}"))
        self._plan_fusions()
        self.training = True
        self.device = torch.device("cpu")

    def _plan_fusions(self):
        # a conv/linear whose producer ends in a plain ReLU fuses that ReLU's backward mask into
        # its dgrad epilogue (dx *= x > 0), the producer then skips its own mask pass.
        for prev, cur in zip(self.layers[:-1], self.layers[1:]):
            if isinstance(cur, ConvUnit) and prev.out_act == RELU and not getattr(prev, "bn", False) \
                    and not getattr(prev, "residual_out", False):
                cur.mask_input = True
                prev.grad_premasked = True
        # residual blocks whose input is relu(BN(c) [+ r]) of the previous layer take over that
        # BN's ReLU mask and backward reduce in their last dgrad epilogue (Layer.fuse_out_bn)
        for prev, cur in zip(self.layers[:-1], self.layers[1:]):
            if getattr(cur, "residual_out", False) and hasattr(cur, "bn_out") \
                    and type(prev).bn_out is not Layer.bn_out and prev.out_act == RELU \
                    and os.environ.get("DDL_FUSE_BN_BWD", "1") != "0":
                cur.fuse_out_bn = True
                prev.accepts_part = True
            # a global average pool after such a block: the pool's backward applies the mask and
            # reduces the block's output BN (one pass instead of pool-bwd + BN reduce)
            if cur.name == "avgpool" and type(prev).bn_out is not Layer.bn_out \
                    and getattr(prev, "residual_out", False) and prev.out_act == RELU \
                    and os.environ.get("DDL_FUSE_BN_BWD", "1") != "0":
                cur.fuse_out_bn = True
                prev.accepts_part = True
        if self.layers:
            self.layers[0].needs_input_grad = False

    # ------------------------------------------------------------------ setup
    @property
    def act_dtype(self):
        return torch.float32 if self.precision == "fp32" else torch.bfloat16

    def _cpu_storage(self):
        """CPU reference ops store activations in the net's precision."""
        if self.device.type == "cpu" and self.precision == "fp32":
            return ref.storage(torch.float32)
        return contextlib.nullcontext()

    def to(self, device, seed: int = 0, generator=None):
        self.device = torch.device(device)
        self.store.materialize(self.device, seed=seed, generator=generator, fp32=self.precision == "fp32")
        for i, layer in enumerate(self.layers):
            layer.bind(self.store)
            if isinstance(layer, Dropout):  # deterministic per (net seed, position)
                layer.seed = (int(seed) * 0x9E3779B97F4A7C15 + i * 0xBF58476D1CE4E5B9) & (2 ** 63 - 1)
                layer.uid = i + 1
        return self

    def rng_counters(self) -> list:
        """Device-resident RNG counters (dropout Philox offsets) — part of the training state."""
        return [layer.ctr for layer in self.layers if isinstance(layer, Dropout) and layer.ctr is not None]

    def train(self, mode: bool = True):
        self.training = mode
        return self

    def eval(self):
        return self.train(False)

    # ------------------------------------------------------------------ native path
    def forward_native(self, x, train: bool | None = None):
        train = self.training if train is None else train
        self.store.ensure_shadow()
        ctxs = []
        with self._cpu_storage():
            for layer in self.layers:
                x, c = layer.forward(x, train)
                ctxs.append(c)
        return x, ctxs

    grad_hook = None  # callable(layer_index) after each layer's weight grads are complete
    # Weight grads on a side stream (Fn.wgrad_overlap). DDL_WGRAD_OVERLAP=1 / 0 forces it; by default
    # it is on for fp32 activations, where it was measured faster on the graph-replayed ResNet-18
    # FedAvg step (1 client 17.97k -> 19.11k, 8 clients 33.9k -> 35.0k samples/s), and off for
    # bf16, where it was measured slower (1 client: 138 -> 152 ms per round). Round 5 (tuned
    # per-client-count plans, scripts/gpu/r5ov.sh): on at 1 / 4 / 8 slots (+0.7 / +0.8 / +1.6 %),
    # off at 2 slots, where it costs 1.4 % (31.4k vs 31.9k samples/s).
    _OVERLAP_ENV = os.environ.get("DDL_WGRAD_OVERLAP", "auto")

    @property
    def overlap_wgrad(self) -> bool:
        forced = self.__dict__.get("_overlap_forced")
        if forced is not None:
            return forced
        if self._OVERLAP_ENV in ("0", "1"):
            return self._OVERLAP_ENV == "1"
        return self.act_dtype == torch.float32 and self.G != 2

    @overlap_wgrad.setter
    def overlap_wgrad(self, on: bool) -> None:
        self.__dict__["_overlap_forced"] = bool(on)

    def backward_native(self, dy, ctxs, part=None):
        """Backward through the first len(ctxs) layers (all of them unless a fused head already
        took the last ones); ``part``: BN backward sums the caller's fused op left for the last of
        those layers."""
        n = len(ctxs)
        with Fn.wgrad_overlap(self.device, self.overlap_wgrad) as ov, self._cpu_storage():
            for j, (layer, c) in enumerate(zip(reversed(self.layers[:n]), reversed(ctxs))):
                i = n - 1 - j
                kw = {"part": part} if part is not None else {}
                fuse = None
                if layer.fuse_out_bn and layer.needs_input_grad and i > 0:
                    fuse = self.layers[i - 1].bn_out(ctxs[i - 1])
                if fuse is not None:
                    kw["fuse"] = fuse
                r = layer.backward(dy, c, **kw)
                dy, part = r if fuse is not None else (r, None)
                if self.grad_hook is not None:
                    # the hook (a bucket all-reduce) must see this layer's grads from both streams
                    ov.run_joined(lambda i=n - 1 - j: self.grad_hook(i))
                if dy is None:
                    break
        return dy

    def train_step(self, x, labels, ncls=None, scale=None, targets=None, with_correct=False):
        """forward + fused softmax-CE (mean over each client's batch) + backward. A net ending in
        global average pool -> Linear runs its head as two fused launches (``Fn.head_train``;
        DDL_FUSED_HEAD=0 keeps the per-layer path). Grads ACCUMULATE into store.grad (zero them
        per optimizer step). Returns (loss[G], correct). The returned loss lives in the step's
        scratch arena: read it before the next step."""
        if not hasattr(self, "_ws"):
            self._ws = Workspace()
        self._ws.begin(self.device)
        self.store.ensure_shadow()  # the fused-head path runs layer.forward itself
        try:
            with self._cpu_storage(), self._presplit(x):
                return self._train_step(x, labels, ncls, scale, targets, with_correct)
        finally:
            self._ws.end()

    def _presplit(self, x):
        """fp32 on the GPU: every X6 weight image of the step in one launch at step start
        (functional_f32.PresplitScope); the weights stay fixed until the step's own updates."""
        if x.is_cuda and self.precision == "fp32":
            return Fn.F32.presplit_scope(self)
        return contextlib.nullcontext()

    def _train_step(self, x, labels, ncls, scale, targets, with_correct):
        head = self._fused_head(x, targets, ncls)
        if head is not None:
            return self._train_step_fused_head(x, labels, head, scale, with_correct)
        logits, ctxs = self.forward_native(x, True)
        N = logits.shape[1]
        loss, dlogits, correct = Fn.cross_entropy(
            logits, labels, targets, ncls=ncls or self.num_classes,
            scale=(1.0 / N) if scale is None else scale, with_correct=with_correct)
        self.backward_native(dlogits, ctxs)
        return loss, correct

    def _fused_head(self, x, targets, ncls):
        """(pool, linear, ncls) when the step can end in ``Fn.head_train``: the net ends in a global
        average pool and a plain Linear (bias or not, no BN / activation), hard labels, on the GPU."""
        if not (x.is_cuda and Fn.HEAD_FUSED and targets is None and len(self.layers) >= 3):
            return None
        pool, lin = self.layers[-2], self.layers[-1]
        if pool.name != "avgpool" or not isinstance(lin, ConvUnit) or not lin.linear or lin.bn or lin.act:
            return None
        ncls = ncls or self.num_classes or lin.cout
        if not Fn.head_train_ok(lin.cin, ncls, x.dtype) or ncls > lin.cout:
            return None
        return pool, lin, ncls

    def _train_step_fused_head(self, x, labels, head, scale, with_correct):
        pool, lin, ncls = head
        ctxs = []
        with self._cpu_storage():
            for layer in self.layers[:-2]:
                x, c = layer.forward(x, True)
                ctxs.append(c)
        st = self.store
        fuse = self.layers[-3].bn_out(ctxs[-1]) if pool.fuse_out_bn else None
        loss, correct, dx, part = Fn.head_train(
            x, st.shadow_of(lin.w), st.param(lin.b) if lin.bias else None,
            labels.to(torch.int32).contiguous(), ncls, (1.0 / x.shape[1]) if scale is None else scale,
            st.grad_of(lin.w), st.grad_of(lin.b) if lin.bias else None, bn=fuse, with_correct=with_correct)
        n = len(self.layers)
        if self.grad_hook is not None:
            self.grad_hook(n - 1)
            self.grad_hook(n - 2)
        self.backward_native(dx, ctxs, part=part)
        return loss, correct

    @torch.no_grad()
    def predict(self, x):
        logits, _ = self.forward_native(x, False)
        return logits

    # ------------------------------------------------------------------ torch-compatible path
    def prepare_input(self, x: torch.Tensor) -> torch.Tensor:
        """Accepts the native layout [G,N,...] in the net's activation dtype, or a torch-style fp32
        batch (NCHW image / [N, F] table) for G == 1, converting it with the kernels' input rules."""
        dt = self.act_dtype
        if x.dtype == dt and x.dim() >= 3 and x.shape[0] == self.G and (dt == torch.bfloat16 or x.dim() != 4):
            return x
        spec = self.input_spec
        if spec.get("flat") and x.dim() > 2:
            x = x.reshape(x.shape[0], -1)
        if x.dim() == 4:  # NCHW images
            return Fn.nchw_to_nhwc(x.to(self.device), spec.get("cpad", 32),
                                   spec.get("stem_k", 0) if spec.get("im2col") else 0,
                                   spec.get("pad", 0), spec.get("stem_stride", 1), dtype=dt)
        if x.dim() == 2:  # [N, F]
            F_ = x.shape[1]
            cp = spec.get("cpad", (F_ + 31) // 32 * 32)
            out = torch.zeros(1, x.shape[0], cp, dtype=dt, device=self.device)
            out[0, :, :F_] = x.to(self.device, dt)
            return out
        raise ValueError(f"unsupported input shape {tuple(x.shape)}")

    def __call__(self, x: torch.Tensor) -> torch.Tensor:
        xin = self.prepare_input(x)
        if torch.is_grad_enabled() and self.training:
            return _NetFunction.apply(self, xin, self._token())
        logits, _ = self.forward_native(xin, self.training)
        return self._logits_out(logits)

    forward = __call__

    def _logits_out(self, logits):
        ncls = self.num_classes or logits.shape[-1]
        out = logits[..., :ncls].float()
        if self.G == 1:
            out = out[0]
        return self.output_transform(out)

    def output_transform(self, logits):
        return logits

    def output_transform_backward(self, out, grad):
        return grad

    def _token(self):
        if not hasattr(self, "_tok"):
            self._tok = torch.zeros((), requires_grad=True)
        return self._tok

    # torch.nn.Module-ish conveniences
    def parameters(self):
        """Flat master buffer (a list carrying ``.store`` so ``optim.SGD(net.parameters())`` works)."""
        return _StoreParams([self.store.data], self.store)

    def zero_grad(self, set_to_none: bool = False):
        self.store.zero_grad()

    def state_dict(self, group: int = 0):
        return self.store.state_dict(group)

    def load_state_dict(self, sd, group=None):
        self.store.load_state_dict(sd, group)

    def num_params(self) -> int:
        return self.store.num_params()


class _StoreParams(list):
    def __init__(self, items, store):
        super().__init__(items)
        self.store = store


class _NetFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, net: Net, xin, token):
        logits, ctxs = net.forward_native(xin, True)
        out = net._logits_out(logits)
        ctx.net, ctx.ctxs, ctx.lshape = net, ctxs, logits.shape
        ctx.save_for_backward(out)
        return out

    @staticmethod
    def backward(ctx, grad):
        net = ctx.net
        (out,) = ctx.saved_tensors
        g = net.output_transform_backward(out, grad.float())
        G, N, ld = ctx.lshape
        full = torch.zeros(G, N, ld, dtype=net.act_dtype, device=g.device)
        ncls = net.num_classes or ld
        full[..., :ncls] = g.reshape(G, N, ncls).to(net.act_dtype)
        net.backward_native(full, ctx.ctxs)
        ctx.ctxs = None
        return None, None, None
