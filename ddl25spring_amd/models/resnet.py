"""ResNet-18 / ResNet-50 (He et al. 2016) on the fused conv/BN kernels, client-batched.

North-star configs (BASELINE.json): "Horizontal FedAvg ResNet-18, CIFAR-10-shape" and
"Data-parallel all-reduce SGD, ResNet-50 ImageNet-shape". Absent from the reference.

MI355X-first choices:
  * the stem's im2col is fused into the device data loader (``ops.prep_images``), so the CIFAR
    stem (3x3, 3->64) and the ImageNet stem (7x7/2, 3->64) run as K=32 / K=160 GEMMs on MFMA
    instead of 3-channel convolutions;
  * BatchNorm statistics come out of the conv epilogue; BN-apply fuses the residual join (identity
    or projected shortcut, whose own BN is folded into the same pass) and the ReLU;
  * backward of the residual join: the shortcut gradient is added inside the dgrad epilogue of
    the block's first conv;
  * fp32 precision (conv_f32.hip): a block's inner BN+ReLU outputs feed only the next conv, so
    they are never stored — that conv applies relu(c * scale + shift) to its operand as it loads
    it (``in_bn``), in the forward and again in its weight-gradient pass.
"""
from __future__ import annotations

import torch

from ..ops import functional as Fn
from ..ops import workspace as ws
from .layers import RELU, ConvUnit, GlobalAvgPool, Layer, Linear, pad32
from .net import Net


class _BNConv(ConvUnit):
    """conv + BN statistics only (activation handled by the enclosing block)."""

    def __init__(self, cin, cout, k, stride, pad):
        super().__init__(cin, cout, k=k, stride=stride, pad=pad, bias=False, bn=True, act=None)

    def conv_raw(self, x, train, in_bn=None):
        """The conv with its BN-statistics epilogue -> (c, stats | None, geom)."""
        g = self.geom(x)
        stats = Fn.stats_buffer(g.G, self.cout, x.device, like=x) if train else None
        return Fn.conv_fwd(x, self.store.shadow_of(self.w), g, stats=stats, in_bn=in_bn), stats, g

    def bn_inputs(self, stats, g):
        st = self.store
        return (stats, st.param(self.gamma), st.param(self.beta), st.buffer(self.rm),
                st.buffer(self.rv), g.N * g.P * g.Q)

    def finalize(self, stats, g, train):
        if not train:
            stats = ws.zeros((g.G, 2, self.cout), self.store.data.device)
        return Fn.bn_finalize(*self.bn_inputs(stats, g), self.eps, self.momentum, training=train)

    def conv_stats(self, x, train, in_bn=None):
        c, stats, g = self.conv_raw(x, train, in_bn)
        sc, sh, mu, rs = self.finalize(stats, g, train)
        return c, sc, sh, mu, rs, g

    def bn_backward(self, dy, ymask, c, mu, rs, emit_dym=False, part=None):
        st = self.store
        return Fn.bn_backward(dy, ymask, c, mu, rs, st.param(self.gamma), st.grad_of(self.gamma),
                              st.grad_of(self.beta), emit_dym=emit_dym, part=part)

    def bn_backward_coef(self, dy, c, mu, rs, part):
        """fp32: this BN's backward without the apply pass -> (c, coef) for conv_dgrad_wgrad(dy_bn=)."""
        st = self.store
        return c, Fn.F32.bn_backward_coef(dy, c, mu, rs, st.param(self.gamma), st.grad_of(self.gamma),
                                          st.grad_of(self.beta), part=part)

    def bn_bwd_inputs(self, c, mu, rs, part):
        st = self.store
        return (c, mu, rs, st.param(self.gamma), st.grad_of(self.gamma), st.grad_of(self.beta), part)


def _conv_pair_bn(main: _BNConv, y, down: _BNConv, x, train, in_bn=None):
    """A block's last conv (on y, or on relu(y * scale + shift) with ``in_bn``) and its projection
    shortcut (on the block input x), as one paired launch where the tuner measured that faster,
    with both BatchNorms finalized in one launch -> (c, bn, g), (cs, bn_s, gs);
    bn = (scale, shift, mean, rstd)."""
    g, gs = main.geom(y), down.geom(x)
    st = Fn.stats_buffer(g.G, main.cout, y.device, like=y) if train else None
    sts = Fn.stats_buffer(gs.G, down.cout, x.device, like=x) if train else None
    if in_bn is not None:
        c = Fn.conv_fwd(y, main.store.shadow_of(main.w), g, stats=st, in_bn=in_bn)
        cs = Fn.conv_fwd(x, down.store.shadow_of(down.w), gs, stats=sts)
    else:
        c, cs = Fn.conv_fwd2(y, main.store.shadow_of(main.w), g, st, x, down.store.shadow_of(down.w), gs, sts)
    if train:
        bn, bns = Fn.bn_finalize2(main.bn_inputs(st, g), down.bn_inputs(sts, gs), main.eps, main.momentum)
    else:
        bn, bns = main.finalize(st, g, train), down.finalize(sts, gs, train)
    return (c, bn, g), (cs, bns, gs)


def _inner_act(c, scale, shift):
    """relu(BN(c)) feeding only the next conv: (activation, None), or in fp32 precision (c, (scale,
    shift)) — the consumer applies it on the fly (operand-side BN), the activation is never stored."""
    if Fn.F32.is_f32(c):
        return c, (scale, shift)
    return Fn.bn_apply(c, scale, shift, act=RELU), None


def _bn_fold(t) -> bool:
    """fp32 activations: BN backwards hand their coefficients to the consuming DGRAD (applied as
    the halo kernel stages dY) instead of running an apply pass (DDL_F32_BNFOLD=0: apply pass)."""
    return Fn.F32.is_f32(t) and Fn.F32.BNFOLD[0]


class _ShortcutGrad:
    def _inner_bn_backward(self, conv, d, c, mu, rs, part, fold):
        """An inner BN's backward -> (operand for the conv's DGRAD/WGRAD, dy_bn or None)."""
        if fold:
            return d, conv.bn_backward_coef(d, c, mu, rs, part)
        return conv.bn_backward(d, None, c, mu, rs, part=part), None

    def _out_and_shortcut_bn_backward(self, main: _BNConv, dout, c, mu, rs, part, dctx):
        """The block's output BN and its shortcut's BN both take the (masked) block output gradient:
        the shortcut's reduce, then ONE fold launch and ONE apply pass for both (bn_backward2).
        -> (d main conv output, d shortcut conv output)."""
        cs, mus, rss, gs = dctx
        part_s = Fn.bn_bwd_reduce_part(dout, None, cs, mus, rss)
        return Fn.bn_backward2(dout, main.bn_bwd_inputs(c, mu, rs, part),
                               self.down.bn_bwd_inputs(cs, mus, rss, part_s))

    def _shortcut_backward(self, dym, dctx, x, dcs=None):
        """Projection shortcut backward: its BN (unless ``dcs`` is given), then its conv's WGRAD
        and (if the block input needs a gradient) DGRAD. A 1x1 / stride-2 shortcut's input
        gradient is nonzero only on the (2i, 2j) pixels, so its DGRAD runs as a dense 1x1 conv on
        the compact grid and the block's first DGRAD adds it there (residual_sub = 2) instead of
        materialising 3/4 zeros. -> (residual for the first conv's DGRAD, residual_sub)."""
        cs, mus, rss, gs = dctx
        st = self.store
        if dcs is None:
            dcs = self.down.bn_backward(dym, None, cs, mus, rss)
        sub = gs.stride == 2 and gs.R == 1 and gs.S == 1 and gs.pad == 0
        dgeom = Fn.ConvGeom(gs.G, gs.N, gs.P, gs.Q, gs.C, gs.K, 1, 1, 1, 0) if sub else None
        dres = Fn.conv_dgrad_wgrad(dcs, st.shadow_of(self.down.w), x, gs, st.grad_of(self.down.w),
                                   want_dx=self.needs_input_grad, dgeom=dgeom)
        return dres, (2 if sub else 1)


class BasicBlock(_ShortcutGrad, Layer):
    name = "basic"
    residual_out = True
    expansion = 1

    def __init__(self, cin, planes, stride=1):
        self.cin, self.cout, self.stride = cin, planes, stride
        self.conv1 = _BNConv(cin, planes, 3, stride, 1)
        self.conv2 = _BNConv(planes, planes, 3, 1, 1)
        self.down = _BNConv(cin, planes, 1, stride, 0) if (stride != 1 or cin != planes) else None

    @property
    def out_act(self):
        return RELU

    def declare(self, store, prefix):
        super().declare(store, prefix)
        self.conv1.declare(store, prefix + ".conv1")
        self.conv2.declare(store, prefix + ".conv2")
        if self.down is not None:
            self.down.declare(store, prefix + ".downsample")

    def bind(self, store):
        super().bind(store)
        for c in (self.conv1, self.conv2, self.down):
            if c is not None:
                c.bind(store)

    def forward(self, x, train):
        c1, sc1, sh1, mu1, rs1, g1 = self.conv1.conv_stats(x, train)
        a1, ib = _inner_act(c1, sc1, sh1)
        if self.down is not None:
            (c2, (sc2, sh2, mu2, rs2), g2), (cs, (scs, shs, mus, rss), gs) = \
                _conv_pair_bn(self.conv2, a1, self.down, x, train, in_bn=ib)
            out = Fn.bn_apply(c2, sc2, sh2, r=cs, rscale=scs, rshift=shs, act=RELU)
            dctx = (cs, mus, rss, gs)
        else:
            c2, sc2, sh2, mu2, rs2, g2 = self.conv2.conv_stats(a1, train, in_bn=ib)
            out = Fn.bn_apply(c2, sc2, sh2, r=x, act=RELU)
            dctx = None
        return out, (x, c1, a1, sc1, sh1, mu1, rs1, g1, c2, mu2, rs2, g2, out, dctx, ib)

    def bn_out(self, ctx):
        return (ctx[8], ctx[9], ctx[10])  # (c2, mu2, rs2): out = relu(bn2(c2) + shortcut)

    def backward(self, dout, ctx, part=None, fuse=None):
        x, c1, a1, sc1, sh1, mu1, rs1, g1, c2, mu2, rs2, g2, out, dctx, ib = ctx
        st = self.store
        dcs = None
        fold = _bn_fold(dout)
        dyb2 = None
        if part is not None and dctx is not None:  # output + shortcut BN backwards together
            (dc2, dcs), dym = self._out_and_shortcut_bn_backward(self.conv2, dout, c2, mu2, rs2, part,
                                                                 dctx), dout
        elif part is not None:  # dout arrives masked by (out > 0) with bn2's reduce sums
            if fold:
                dc2, dyb2 = dout, self.conv2.bn_backward_coef(dout, c2, mu2, rs2, part)
            else:
                dc2 = self.conv2.bn_backward(dout, None, c2, mu2, rs2, part=part)
            dym = dout
        else:
            dc2, dym = self.conv2.bn_backward(dout, out, c2, mu2, rs2, emit_dym=True)
        # every conv's DGRAD and WGRAD read the same dY: one (possibly paired) launch each
        dres, rsub = self._shortcut_backward(dym, dctx, x, dcs) if dctx is not None else (dym, 1)
        # dgrad epilogue applies bn1's ReLU mask (recomputed from c1: no read of a1) and reduces
        # bn1's backward sums (no reduce pass)
        da1, part1 = Fn.conv_dgrad_wgrad(dc2, st.shadow_of(self.conv2.w), a1, g2, st.grad_of(self.conv2.w),
                                         bn=(c1, mu1, rs1), mask_bn=(sc1, sh1), in_bn=ib, dy_bn=dyb2)
        dc1, dyb1 = self._inner_bn_backward(self.conv1, da1, c1, mu1, rs1, part1, fold)
        # with fuse: the producer's ReLU mask (x > 0) and BN reduce in this dgrad's epilogue
        return Fn.conv_dgrad_wgrad(dc1, st.shadow_of(self.conv1.w), x, g1, st.grad_of(self.conv1.w),
                                   residual=dres, mask=x if fuse is not None else None, bn=fuse,
                                   want_dx=self.needs_input_grad, residual_sub=rsub, dy_bn=dyb1)

    def flops(self, s):
        G, N, H, W, _ = s
        Ho, Wo = (H + 2 - 3) // self.stride + 1, (W + 2 - 3) // self.stride + 1
        f = 2 * G * N * Ho * Wo * self.cout * 9 * (self.cin + self.cout)
        if self.down is not None:
            f += 2 * G * N * Ho * Wo * self.cout * self.cin
        return f

    def out_shape(self, s):
        G, N, H, W, _ = s
        return (G, N, (H + 2 - 3) // self.stride + 1, (W + 2 - 3) // self.stride + 1, self.cout)


class Bottleneck(_ShortcutGrad, Layer):
    name = "bottleneck"
    residual_out = True
    expansion = 4

    def __init__(self, cin, planes, stride=1):
        self.cin, self.cout, self.stride = cin, planes * 4, stride
        self.conv1 = _BNConv(cin, planes, 1, 1, 0)
        self.conv2 = _BNConv(planes, planes, 3, stride, 1)
        self.conv3 = _BNConv(planes, planes * 4, 1, 1, 0)
        self.down = _BNConv(cin, planes * 4, 1, stride, 0) if (stride != 1 or cin != planes * 4) else None
        self.planes = planes

    @property
    def out_act(self):
        return RELU

    def declare(self, store, prefix):
        super().declare(store, prefix)
        for n in ("conv1", "conv2", "conv3"):
            getattr(self, n).declare(store, f"{prefix}.{n}")
        if self.down is not None:
            self.down.declare(store, prefix + ".downsample")

    def bind(self, store):
        super().bind(store)
        for c in (self.conv1, self.conv2, self.conv3, self.down):
            if c is not None:
                c.bind(store)

    def forward(self, x, train):
        c1, sc1, sh1, mu1, rs1, g1 = self.conv1.conv_stats(x, train)
        a1, ib1 = _inner_act(c1, sc1, sh1)
        c2, sc2, sh2, mu2, rs2, g2 = self.conv2.conv_stats(a1, train, in_bn=ib1)
        a2, ib2 = _inner_act(c2, sc2, sh2)
        if self.down is not None:
            (c3, (sc3, sh3, mu3, rs3), g3), (cs, (scs, shs, mus, rss), gs) = \
                _conv_pair_bn(self.conv3, a2, self.down, x, train, in_bn=ib2)
            out = Fn.bn_apply(c3, sc3, sh3, r=cs, rscale=scs, rshift=shs, act=RELU)
            dctx = (cs, mus, rss, gs)
        else:
            c3, sc3, sh3, mu3, rs3, g3 = self.conv3.conv_stats(a2, train, in_bn=ib2)
            out = Fn.bn_apply(c3, sc3, sh3, r=x, act=RELU)
            dctx = None
        return out, (x, (c1, a1, sc1, sh1, mu1, rs1, g1), (c2, a2, sc2, sh2, mu2, rs2, g2),
                     (c3, mu3, rs3, g3), out, dctx, (ib1, ib2))

    def bn_out(self, ctx):
        return ctx[3][:3]  # (c3, mu3, rs3): out = relu(bn3(c3) + shortcut)

    def backward(self, dout, ctx, part=None, fuse=None):
        x, (c1, a1, sc1, sh1, mu1, rs1, g1), (c2, a2, sc2, sh2, mu2, rs2, g2), (c3, mu3, rs3, g3), out, dctx, \
            (ib1, ib2) = ctx
        st = self.store
        dcs = None
        fold = _bn_fold(dout)
        dyb3 = None
        if part is not None and dctx is not None:  # output + shortcut BN backwards together
            (dc3, dcs), dym = self._out_and_shortcut_bn_backward(self.conv3, dout, c3, mu3, rs3, part,
                                                                 dctx), dout
        elif part is not None:  # dout arrives masked by (out > 0) with bn3's reduce sums
            if fold:
                dc3, dyb3 = dout, self.conv3.bn_backward_coef(dout, c3, mu3, rs3, part)
            else:
                dc3 = self.conv3.bn_backward(dout, None, c3, mu3, rs3, part=part)
            dym = dout
        else:
            dc3, dym = self.conv3.bn_backward(dout, out, c3, mu3, rs3, emit_dym=True)
        dres, rsub = self._shortcut_backward(dym, dctx, x, dcs) if dctx is not None else (dym, 1)
        da2, part2 = Fn.conv_dgrad_wgrad(dc3, st.shadow_of(self.conv3.w), a2, g3, st.grad_of(self.conv3.w),
                                         bn=(c2, mu2, rs2), mask_bn=(sc2, sh2), in_bn=ib2, dy_bn=dyb3)
        dc2, dyb2 = self._inner_bn_backward(self.conv2, da2, c2, mu2, rs2, part2, fold)
        da1, part1 = Fn.conv_dgrad_wgrad(dc2, st.shadow_of(self.conv2.w), a1, g2, st.grad_of(self.conv2.w),
                                         bn=(c1, mu1, rs1), mask_bn=(sc1, sh1), in_bn=ib1, dy_bn=dyb2)
        dc1, dyb1 = self._inner_bn_backward(self.conv1, da1, c1, mu1, rs1, part1, fold)
        return Fn.conv_dgrad_wgrad(dc1, st.shadow_of(self.conv1.w), x, g1, st.grad_of(self.conv1.w),
                                   residual=dres, mask=x if fuse is not None else None, bn=fuse,
                                   want_dx=self.needs_input_grad, residual_sub=rsub, dy_bn=dyb1)

    def flops(self, s):
        G, N, H, W, _ = s
        Ho, Wo = (H + 2 - 3) // self.stride + 1, (W + 2 - 3) // self.stride + 1
        p = self.planes
        f = 2 * G * N * (H * W * p * self.cin + Ho * Wo * p * 9 * p + Ho * Wo * self.cout * p)
        if self.down is not None:
            f += 2 * G * N * Ho * Wo * self.cout * self.cin
        return f

    def out_shape(self, s):
        G, N, H, W, _ = s
        return (G, N, (H + 2 - 3) // self.stride + 1, (W + 2 - 3) // self.stride + 1, self.cout)


class MaxPool3s2(Layer):
    """3x3/2 pad-1 max pool of the ImageNet stem (via two 2x2 reductions is NOT equivalent, so it
    runs as its own kernel)."""
    name = "maxpool3"

    def forward(self, x, train):
        if not train:
            return Fn.maxpool_fwd(x, 3, 2, 1), None
        y, am = Fn.maxpool_fwd(x, 3, 2, 1, want_argmax=True)
        return y, (x, am)

    def backward(self, dy, ctx):
        x, am = ctx
        return Fn.maxpool_bwd(x, dy, 3, 2, 1, argmax=am)

    def out_shape(self, s):
        G, N, H, W, C = s
        return (G, N, (H + 2 - 3) // 2 + 1, (W + 2 - 3) // 2 + 1, C)


def _resnet(block, layers, num_classes, groups, stem: str, in_ch=3, precision=None) -> Net:
    mods: list[Layer] = []
    if stem == "cifar":
        # im2col'd 3x3 stem: channel j = (r*3+s)*3 + c (27 real of 32), 1x1 conv on MFMA
        stem_conv = ConvUnit(32, 64, k=1, stride=1, pad=0, bn=True, act="relu",
                             cin_true=9 * in_ch, fan_in=9 * in_ch)
        input_spec = {"cpad": 32, "im2col": True, "pad": 1, "stem_k": 3}
    else:
        cpad = pad32(49 * in_ch)
        stem_conv = ConvUnit(cpad, 64, k=1, stride=1, pad=0, bn=True, act="relu",
                             cin_true=49 * in_ch, fan_in=49 * in_ch)
        input_spec = {"cpad": cpad, "im2col": True, "pad": 3, "stem_k": 7, "stem_stride": 2}
    stem_conv.pname = "conv1"
    mods.append(stem_conv)
    if stem != "cifar":
        mp = MaxPool3s2()
        mp.pname = "maxpool"
        mods.append(mp)
    cin = 64
    for li, (planes, n) in enumerate(zip((64, 128, 256, 512), layers)):
        for bi in range(n):
            stride = 2 if (bi == 0 and li > 0) else 1
            b = block(cin, planes, stride)
            b.pname = f"layer{li + 1}.{bi}"
            mods.append(b)
            cin = planes * block.expansion
    gp = GlobalAvgPool()
    gp.pname = "avgpool"
    mods.append(gp)
    fc = Linear(cin, num_classes, bias=True, fout_true=num_classes)
    fc.pname = "fc"
    mods.append(fc)
    net = Net(mods, groups=groups, num_classes=num_classes, input_spec=input_spec,
              name=f"resnet{sum(layers) * (2 if block is BasicBlock else 3) + 2}", precision=precision)
    return net


def resnet18_cifar(num_classes=10, groups=1, precision=None) -> Net:
    """ResNet-18, CIFAR variant (3x3 stem, no max-pool), 11.17M params."""
    return _resnet(BasicBlock, (2, 2, 2, 2), num_classes, groups, "cifar", precision=precision)


def resnet50_imagenet(num_classes=1000, groups=1, precision=None) -> Net:
    """ResNet-50, ImageNet variant (7x7/2 stem + 3x3/2 max-pool), 25.6M params."""
    return _resnet(Bottleneck, (3, 4, 6, 3), num_classes, groups, "imagenet", precision=precision)


def resnet18_imagenet(num_classes=1000, groups=1, precision=None) -> Net:
    return _resnet(BasicBlock, (2, 2, 2, 2), num_classes, groups, "imagenet", precision=precision)
