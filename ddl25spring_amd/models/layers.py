"""Explicit forward/backward layers over the HIP op layer, with a leading client-group dim.

The framework does not route its hot path through the autograd engine: each layer saves exactly
what its backward needs and calls fused kernels (conv epilogue BN-statistics, BN+residual+ReLU
apply, ReLU masks fused into the next layer's dgrad epilogue, weight grads accumulated straight
into the flat fp32 grad buffer). A whole model can still be used as a single autograd node
(:class:`ddl25spring_amd.models.net.Net` wraps it) so notebook-style code
``loss.backward(); optimizer.step()`` keeps working.

Activation shapes: ``[G, N, H, W, C]`` (spatial) or ``[G, N, C]`` (dense), bf16, channels padded
to multiples of 32 (the MFMA K granule).
"""
from __future__ import annotations

import math

import torch

from ..ops import functional as Fn
from ..ops import workspace as ws
from ..ops.functional import ConvGeom
from .params import ParamStore, const_, kaiming_uniform_, uniform_bias_

RELU, LEAKY = 1, 2
_ACT = {None: 0, "none": 0, "relu": RELU, "leaky_relu": LEAKY}


def pad32(n: int) -> int:
    return (n + 31) // 32 * 32


class Layer:
    """Base: declare params -> bind views -> forward(x) -> (y, ctx) -> backward(dy, ctx) -> dx."""
    name = "layer"
    # set by Net when the producer of this layer's input applies a ReLU that this layer's dgrad
    # epilogue can fuse (dx *= (x > 0)).
    mask_input = False
    # set by Net when the next layer already applied this layer's output activation mask.
    grad_premasked = False
    needs_input_grad = True
    # Cross-layer BN-backward fusion (Net._plan_fusions): a layer whose output is
    # relu(BN(c) [+ residual]) exposes (c, mean, rstd) via ``bn_out``; the consuming layer's final
    # dgrad (``fuse_out_bn``) then applies that ReLU mask and reduces the BN's backward sums in its
    # epilogue and returns (dx_masked, part); the producer's ``backward(..., part=part)`` skips its
    # reduce pass, the mask read and the masked-gradient copy.
    fuse_out_bn = False
    accepts_part = False

    def bn_out(self, ctx):
        return None

    def declare(self, store: ParamStore, prefix: str) -> None:
        self.prefix = prefix

    def bind(self, store: ParamStore) -> None:
        self.store = store

    def forward(self, x, train: bool):
        raise NotImplementedError

    def backward(self, dy, ctx):
        raise NotImplementedError

    @property
    def out_act(self) -> int:
        return 0

    def flops(self, x_shape) -> int:
        return 0


class ConvUnit(Layer):
    """conv(KxRxS) [+ bias | + BatchNorm(batch stats)] [+ act]; Linear is the 1x1-on-1x1 case.

    ``cin`` is the padded input channel count seen by the kernel; ``cin_true`` the real one (the
    rest is zero data, e.g. the stem im2col channels). ``cout`` is padded to 32 (zero rows).
    """

    def __init__(self, cin, cout, k=3, stride=1, pad=None, bias=False, bn=False, act=None,
                 cin_true=None, cout_true=None, fan_in=None, bn_eps=1e-5, bn_momentum=0.1,
                 linear=False):
        self.cin, self.cout = pad32(cin), pad32(cout)
        self.cin_true = cin_true if cin_true is not None else cin
        self.cout_true = cout_true if cout_true is not None else cout
        self.k, self.stride = k, stride
        self.pad = (k // 2) if pad is None else pad
        self.bias, self.bn, self.act = bias, bn, _ACT[act]
        self.fan_in = fan_in if fan_in is not None else self.cin_true * k * k
        self.eps, self.momentum = bn_eps, bn_momentum
        self.linear = linear
        self.name = "linear" if linear else "conv"

    @property
    def out_act(self):
        return self.act

    def declare(self, store, prefix):
        super().declare(store, prefix)
        p = prefix
        shape = (self.cout, self.k, self.k, self.cin)
        init_w = kaiming_uniform_(self.fan_in)
        cin_t, cout_t, k = self.cin_true, self.cout_true, self.k

        def winit(t, gen, init_w=init_w):
            t.zero_()
            # draw in torch's [out, in, kh, kw] order, then lay out as [out, kh, kw, in]
            w = torch.empty(cout_t, cin_t, k, k)
            init_w(w, gen)
            t[:cout_t, :, :, :cin_t] = w.permute(0, 2, 3, 1)
        # every conv weight takes direct SGD; Linear weights unless Net marked the layer a fused
        # classifier head (its weight gradient comes from Fn.head_train, not a WGRAD launch)
        self.w = store.add(p + ".weight", shape, winit,
                           direct=not self.linear or getattr(self, "direct_w", False))
        if self.bias:
            binit = uniform_bias_(self.fan_in)

            def bi(t, gen, binit=binit):
                t.zero_()
                b = torch.empty(cout_t)
                binit(b, gen)
                t[:cout_t] = b
            self.b = store.add(p + ".bias", (self.cout,), bi)
        if self.bn:
            def gi(t, gen):
                t.zero_()
                t[:cout_t] = 1.0
            self.gamma = store.add(p + ".bn.weight", (self.cout,), gi)
            self.beta = store.add(p + ".bn.bias", (self.cout,), const_(0.0))
            self.rm = store.add(p + ".bn.running_mean", (self.cout,), const_(0.0), buffer=True)
            self.rv = store.add(p + ".bn.running_var", (self.cout,), const_(1.0), buffer=True)

    def geom(self, x) -> ConvGeom:
        if self.linear:
            G, N = x.shape[0], x.shape[1]
            return ConvGeom(G, N, 1, 1, self.cin, self.cout, 1, 1, 1, 0)
        G, N, H, W, C = x.shape
        return ConvGeom(G, N, H, W, C, self.cout, self.k, self.k, self.stride, self.pad)

    def _x4(self, x):
        return x.reshape(x.shape[0], x.shape[1], 1, 1, x.shape[-1]) if self.linear else x

    def forward(self, x, train):
        st = self.store
        assert x.shape[-1] == self.cin, f"{self.prefix}: got C={x.shape[-1]}, want {self.cin}"
        x4 = self._x4(x)
        g = self.geom(x4)
        w = st.shadow_of(self.w)
        if self.bn:
            stats = Fn.stats_buffer(g.G, self.cout, x.device, like=x) if train else None
            c = Fn.conv_fwd(x4, w, g, stats=stats)
            count = g.N * g.P * g.Q
            sc, sh, mu, rs = Fn.bn_finalize(stats if train else Fn.stats_buffer(g.G, self.cout, x.device),
                                            st.param(self.gamma), st.param(self.beta),
                                            st.buffer(self.rm), st.buffer(self.rv), count,
                                            self.eps, self.momentum, training=train)
            y = Fn.bn_apply(c, sc, sh, act=self.act)
            ctx = (x4, c, y, mu, rs, g)
        else:
            b = st.param(self.b) if self.bias else None
            y = Fn.conv_fwd(x4, w, g, bias=b, relu=(self.act == RELU))
            if self.act == LEAKY:
                y = Fn.act_fwd(y, LEAKY)
            ctx = (x4, None, y, None, None, g)
        if self.linear:
            y = y.reshape(g.G, g.N, self.cout)
        return y, ctx

    def bn_out(self, ctx):
        return (ctx[1], ctx[3], ctx[4]) if (self.bn and self.act == RELU and not self.linear) else None

    def backward(self, dy, ctx, part=None):
        st = self.store
        x4, c, y, mu, rs, g = ctx
        dy = dy.reshape(y.shape)
        if self.bn:
            premasked = self.grad_premasked or part is not None
            ymask = y if (self.act == RELU and not premasked) else None
            if self.act == LEAKY and not premasked:
                dy = Fn.act_bwd(y, dy, LEAKY)
            dc = Fn.bn_backward(dy, ymask, c, mu, rs, st.param(self.gamma), st.grad_of(self.gamma),
                                st.grad_of(self.beta), part=part)
        else:
            dc = dy
            if self.act and not self.grad_premasked:
                dc = Fn.act_bwd(y, dy, self.act)
            if self.bias:
                Fn.channel_sum(dc, st.grad_of(self.b))
        # DGRAD before WGRAD: in fp32 precision the DGRAD reads the master weight itself, which a
        # direct-SGD WGRAD (ParamStore.direct_update) steps in place
        dx = None
        if self.needs_input_grad:
            dx = Fn.conv_dgrad(dc, st.shadow_of(self.w), g, mask=x4 if self.mask_input else None)
            if self.linear:
                dx = dx.reshape(g.G, g.N, self.cin)
        Fn.conv_wgrad(dc, x4, g, st.grad_of(self.w))
        return dx

    def flops(self, x_shape):
        if self.linear:
            return 2 * x_shape[0] * x_shape[1] * self.cin_true * self.cout_true
        G, N, H, W, _ = x_shape
        P = (H + 2 * self.pad - self.k) // self.stride + 1
        Q = (W + 2 * self.pad - self.k) // self.stride + 1
        return 2 * G * N * P * Q * self.cout_true * self.k * self.k * self.cin_true


def Linear(fin, fout, bias=True, act=None, bn=False, fin_true=None, fout_true=None, **kw):
    return ConvUnit(fin, fout, k=1, stride=1, pad=0, bias=bias, bn=bn, act=act,
                    cin_true=fin_true if fin_true is not None else fin,
                    cout_true=fout_true if fout_true is not None else fout, linear=True, **kw)


class Activation(Layer):
    name = "act"

    def __init__(self, act):
        self.act = _ACT[act]

    @property
    def out_act(self):
        return self.act

    def forward(self, x, train):
        y = Fn.act_fwd(x, self.act)
        return y, y

    def backward(self, dy, y):
        return dy if self.grad_premasked else Fn.act_bwd(y, dy, self.act)


class MaxPool2(Layer):
    name = "maxpool2"

    def forward(self, x, train):
        return Fn.maxpool2_fwd(x), x

    def backward(self, dy, x):
        return Fn.maxpool2_bwd(x, dy)


class GlobalAvgPool(Layer):
    name = "avgpool"

    def forward(self, x, train):
        return Fn.avgpool_fwd(x), (x.shape[2], x.shape[3], x)

    def backward(self, dy, ctx, fuse=None):
        H, W, x = ctx
        if fuse is not None:  # the producer's output ReLU mask + BN backward reduce (Net fusion)
            return Fn.avgpool_bwd_bn(dy, x, fuse)
        return Fn.avgpool_bwd(dy, H, W)


class Flatten(Layer):
    """NHWC flatten: [G,N,H,W,C] -> [G,N,H*W*C] (a view; torch's NCHW flatten order is handled by
    the weight import of the following Linear)."""
    name = "flatten"

    def forward(self, x, train):
        return x.reshape(x.shape[0], x.shape[1], -1), x.shape

    def backward(self, dy, shape):
        return dy.reshape(shape)


class Dropout(Layer):
    """Philox dropout whose counter lives on the device: forward and backward of a step share
    the mask, ``backward`` advances the counter by a stream-ordered kernel, so HIP-graph replays
    draw fresh masks and two nets built with the same seed draw identical ones (the seed comes
    from the net seed and the layer's position, set in ``Net.to``)."""
    name = "dropout"

    def __init__(self, p):
        self.p = float(p)
        self.seed = 0x5EED
        self.uid = 1
        self.ctr = None

    def bind(self, store) -> None:
        super().bind(store)
        self.ctr = torch.zeros(1, dtype=torch.int64, device=store.data.device)

    def forward(self, x, train):
        if not train or self.p <= 0:
            return x, None
        off = self.uid << 40
        return Fn.dropout(x, self.p, self.seed, off, self.ctr), off

    def backward(self, dy, off):
        if off is None:
            return dy
        dx = Fn.dropout(dy.contiguous(), self.p, self.seed, off, self.ctr)
        Fn.u64_add(self.ctr, dy.numel())
        return dx


def fan_in_of(layer: ConvUnit) -> int:
    return layer.cin_true * layer.k * layer.k


def conv_out(h, k, s, p):
    return (h + 2 * p - k) // s + 1


def num_flops(layers, x_shape) -> int:
    tot = 0
    shape = tuple(x_shape)
    for layer in layers:
        tot += layer.flops(shape)
        shape = out_shape(layer, shape)
    return tot


def out_shape(layer, shape):
    if isinstance(layer, ConvUnit):
        if layer.linear:
            return (shape[0], shape[1], layer.cout)
        G, N, H, W, _ = shape
        return (G, N, conv_out(H, layer.k, layer.stride, layer.pad),
                conv_out(W, layer.k, layer.stride, layer.pad), layer.cout)
    if isinstance(layer, MaxPool2):
        G, N, H, W, C = shape
        return (G, N, H // 2, W // 2, C)
    if isinstance(layer, GlobalAvgPool):
        return (shape[0], shape[1], shape[-1])
    if isinstance(layer, Flatten):
        return (shape[0], shape[1], math.prod(shape[2:]))
    if hasattr(layer, "out_shape"):
        return layer.out_shape(shape)
    return shape
