"""Client-batched (grouped) autograd ops: G clients' copies of a layer run as ONE launch.

Activations carry a leading group dim ``[G, N, ...]`` (G = client slots in use); a parameter is a
slot tensor ``[S, ...]`` (S >= G; optim.SlotAdam's strided row views) of which rows 0..G-1 are
used. On the device every op is the grouped form of the ``autograd_ops`` kernel (the native conv /
BN kernels are client-batched through their group dim); weight gradients accumulate straight into
the slot rows of the parameter's gradient (``_ddl_fuse_grad``) or come back as a full [S, ...]
gradient. On the CPU each op loops over the groups with plain PyTorch (the numerics reference).

Precision follows the activations: fp32 inputs (the default, the reference's precision) run every
op on the fp32 kernels (conv_f32.hip, bn_f32.hip, the deterministic fp32 BCE) with the fp32 slot
rows of the parameters as operands; bf16 inputs run the bf16 MFMA kernels on the bf16 shadow rows.

Used by the client-batched federated DCGAN (fl/gan.py; reference aggregation template
lab/tutorial_1a/hfl_complete.py:336-390; the generative lab trains fp32,
lab/tutorial_2a/generative-modeling.py:13-130).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import functional as Fn

_BN_ACT = {"none": 0, "relu": 1, "leaky_relu": 3}


def _sink(p, G):
    if getattr(p, "_ddl_fuse_grad", False) and p.grad is not None and p.grad.dtype == torch.float32:
        return p.grad[:G]
    return None


def _full(p, G, rows):
    """A [S, ...] gradient holding ``rows`` ([G, ...]) in its first G rows."""
    out = torch.zeros(p.shape, dtype=torch.float32, device=rows.device)
    out[:G] = rows.view(G, *p.shape[1:])
    return out


def _wb(w, G, dtype=torch.bfloat16):
    """The first G slot rows of a weight as the kernel operand: the fp32 master rows themselves
    (strided rows of SlotAdam's buffer; the fp32 kernels take a group stride) or the bf16 shadow."""
    if dtype == torch.float32:
        return w.detach()[:G]
    sh = getattr(w, "_ddl_bf16", None)
    if sh is not None:
        return sh[:G]
    return Fn.to_bf16(w.detach()[:G].contiguous())


def _act(t, dtype=None):
    """An activation in the op's precision: ``dtype`` if given, else its own (fp32 or bf16)."""
    if dtype is None:
        dtype = t.dtype if t.dtype in (torch.float32, torch.bfloat16) else torch.bfloat16
    return t.to(dtype).contiguous()


_bf = _act


# ----------------------------------------------------------------------------------- conv
class _GConv2d(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, stride, pad, want_stats):
        G, N, H, W, C = x.shape
        _, Kc, R, S, _ = w.shape
        g = Fn.ConvGeom(G, N, H, W, C, Kc, R, S, stride, pad)
        wb = _wb(w, G, x.dtype)
        stats = Fn.stats_buffer(G, Kc, x.device, like=x) if want_stats else None
        y = Fn.conv_fwd(x, wb, g, stats=stats)
        ctx.save_for_backward(x, wb)
        ctx.g, ctx.w = g, w
        if want_stats and torch.is_tensor(stats):
            ctx.mark_non_differentiable(stats)
        return y.view(G, N, g.P, g.Q, Kc), stats

    @staticmethod
    def backward(ctx, dy, _dstats):
        x, wb = ctx.saved_tensors
        g = ctx.g
        dy5 = _act(dy, x.dtype).view(g.G, g.N, g.P, g.Q, g.K)
        dx = dw = None
        if ctx.needs_input_grad[1]:
            sink = _sink(ctx.w, g.G)
            dwt = sink if sink is not None else torch.zeros(g.G, g.K, g.R, g.S, g.C, dtype=torch.float32,
                                                            device=dy.device)
            dx = Fn.conv_dgrad_wgrad(dy5, wb, x, g, dwt, want_dx=ctx.needs_input_grad[0])
            dw = None if sink is not None else _full(ctx.w, g.G, dwt)
        elif ctx.needs_input_grad[0]:
            dx = Fn.conv_dgrad(dy5, wb, g)
        return dx, dw, None, None, None


def conv2d(x, w, stride=1, pad=0, with_stats=False):
    """x [G, N, H, W, C] NHWC, w [S, K, R, S, C] -> [G, N, P, Q, K] (+ BN statistics)."""
    G = x.shape[0]
    if not x.is_cuda:
        ys = [F.conv2d(x[g].permute(0, 3, 1, 2), w[g].permute(0, 3, 1, 2), stride=stride, padding=pad)
              .permute(0, 2, 3, 1) for g in range(G)]
        y = torch.stack(ys)
        return (y, None) if with_stats else y
    y, st = _GConv2d.apply(_act(x), w, stride, pad, with_stats)
    return (y, st) if with_stats else y


class _GConvT2d(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, stride, pad):
        G, N, Hi, Wi, _ = x.shape
        _, Cin, R, S, Cout = w.shape
        Ho, Wo = (Hi - 1) * stride - 2 * pad + R, (Wi - 1) * stride - 2 * pad + S
        g = Fn.ConvGeom(G, N, Ho, Wo, Cout, Cin, R, S, stride, pad)  # the conv this one transposes
        assert (g.P, g.Q) == (Hi, Wi), "transposed conv geometry must invert exactly"
        wb = _wb(w, G, x.dtype)
        y = Fn.conv_dgrad(x, wb, g)
        ctx.save_for_backward(x, wb)
        ctx.g, ctx.w = g, w
        return y.view(G, N, Ho, Wo, Cout)

    @staticmethod
    def backward(ctx, dy):
        x, wb = ctx.saved_tensors
        g = ctx.g
        dy5 = _act(dy, x.dtype).view(g.G, g.N, g.H, g.W, g.C)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = Fn.conv_fwd(dy5, wb, g).view(x.shape)
        if ctx.needs_input_grad[1]:
            sink = _sink(ctx.w, g.G)
            dwt = sink if sink is not None else torch.zeros(g.G, g.K, g.R, g.S, g.C, dtype=torch.float32,
                                                            device=dy.device)
            Fn.conv_wgrad(x, dy5, g, dwt)
            dw = None if sink is not None else _full(ctx.w, g.G, dwt)
        return dx, dw, None, None


def conv_transpose2d(x, w, stride=1, pad=0):
    """x [G, N, Hi, Wi, Cin], w [S, Cin, R, S, Cout] (nn.ConvTranspose2d, no bias)."""
    G = x.shape[0]
    if not x.is_cuda:
        return torch.stack([F.conv_transpose2d(x[g].permute(0, 3, 1, 2), w[g].permute(0, 3, 1, 2), stride=stride,
                                               padding=pad).permute(0, 2, 3, 1) for g in range(G)])
    return _GConvT2d.apply(_act(x), w, stride, pad)


# --------------------------------------------------------------------------------- linear
class _GLinear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w):
        G, N, C = x.shape
        Kout = w.shape[1]
        g = Fn.ConvGeom(G, N, 1, 1, C, Kout, 1, 1, 1, 0)
        wb = _wb(w, G, x.dtype).view(G, Kout, 1, 1, C)
        y = Fn.conv_fwd(x.view(G, N, 1, 1, C), wb, g)
        ctx.save_for_backward(x, wb)
        ctx.g, ctx.w = g, w
        return y.view(G, N, Kout)

    @staticmethod
    def backward(ctx, dy):
        x, wb = ctx.saved_tensors
        g = ctx.g
        dy5 = _act(dy, x.dtype).view(g.G, g.N, 1, 1, g.K)
        dx = dw = None
        if ctx.needs_input_grad[1]:
            sink = _sink(ctx.w, g.G)
            dwt = sink.view(g.G, g.K, 1, 1, g.C) if sink is not None else \
                torch.zeros(g.G, g.K, 1, 1, g.C, dtype=torch.float32, device=dy.device)
            dx = Fn.conv_dgrad_wgrad(dy5, wb, x.view(g.G, g.N, 1, 1, g.C), g, dwt,
                                     want_dx=ctx.needs_input_grad[0])
            dw = None if sink is not None else _full(ctx.w, g.G, dwt)
        elif ctx.needs_input_grad[0]:
            dx = Fn.conv_dgrad(dy5, wb, g)
        if dx is not None:
            dx = dx.view(g.G, g.N, g.C)
        return dx, dw


def linear(x, w):
    """x [G, N, C], w [S, K, C] -> [G, N, K] (no bias)."""
    G = x.shape[0]
    if not x.is_cuda:
        return torch.stack([x[g] @ w[g].t() for g in range(G)])
    return _GLinear.apply(_act(x), w)


# ------------------------------------------------------------------------------ batchnorm
class _GBatchNormAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, running_mean, running_var, stats, training, momentum, eps, act):
        G, C = x.shape[0], x.shape[-1]
        xg = x.contiguous().view(G, -1, C)
        M = xg.shape[1]
        if training and stats is None:
            stats = Fn.bn_stats(xg)
        if stats is None:
            stats = torch.zeros(G, 2, C, dtype=torch.float32, device=x.device)
        ga, be = gamma.detach()[:G], beta.detach()[:G]
        if not (Fn.F32.is_f32(xg) and ga.stride(-1) == 1 and be.stride(-1) == 1 and ga.stride(0) == be.stride(0)):
            # the fp32 BN kernels take the slot rows in place (one group stride for gamma and beta:
            # rows of SlotAdam's flat buffer); otherwise compact copies
            ga, be = ga.contiguous(), be.contiguous()
        rm, rv = running_mean[:G], running_var[:G]
        scale, shift, mean, rstd = Fn.bn_finalize(stats, ga, be, rm, rv, M, eps, momentum, training)
        y = Fn.bn_apply(xg, scale, shift, act=_BN_ACT[act])
        ctx.save_for_backward(xg, y, mean, rstd, ga)
        ctx.act, ctx.shape, ctx.params = act, x.shape, (gamma, beta)
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, dy):
        xg, y, mean, rstd, ga = ctx.saved_tensors
        G, C = xg.shape[0], xg.shape[-1]
        d = _act(dy, xg.dtype).view_as(xg)
        ymask = None
        if ctx.act == "relu":
            ymask = y
        elif ctx.act == "leaky_relu":
            d = Fn.act_bwd(y, d, 2, 0.2)
        sg, sb = (_sink(p, G) for p in ctx.params)
        if sg is not None and sb is not None and sg.stride(0) == sb.stride(0) == ga.stride(0) \
                and sg.stride(-1) == 1 and sb.stride(-1) == 1:
            # the kernel accumulates d(gamma), d(beta) into the gradient's slot rows: bitwise the
            # zero-filled temporaries plus add_ it replaces (0 + s is exact), four launches fewer
            dx = Fn.bn_backward(d, ymask, xg, mean, rstd, ga, sg, sb)
            return dx.view(ctx.shape), None, None, None, None, None, None, None, None, None
        if ga.stride(0) != C:
            ga = ga.contiguous()
        dgamma = torch.zeros(G, C, dtype=torch.float32, device=dy.device)
        dbeta = torch.zeros(G, C, dtype=torch.float32, device=dy.device)
        dx = Fn.bn_backward(d, ymask, xg, mean, rstd, ga, dgamma, dbeta)
        outs = []
        for p, d_ in zip(ctx.params, (dgamma, dbeta)):
            sink = _sink(p, G)
            if sink is not None:
                sink.add_(d_)
                outs.append(None)
            else:
                outs.append(_full(p, G, d_))
        return dx.view(ctx.shape), outs[0], outs[1], None, None, None, None, None, None, None


def batch_norm_act(x, gamma, beta, running_mean, running_var, training=True, momentum=0.1, eps=1e-5,
                   act="none", stats=None):
    """Per-group BatchNorm over all but the channel dim of x [G, ..., C] (+ fused activation);
    gamma / beta / running stats are [S, C] slot tensors."""
    G, C = x.shape[0], x.shape[-1]
    if not x.is_cuda:
        ys = []
        for g in range(G):
            y = F.batch_norm(x[g].reshape(-1, C), running_mean[g], running_var[g], gamma[g], beta[g], training,
                             momentum, eps).view(x.shape[1:])
            ys.append({"none": y, "relu": F.relu(y), "leaky_relu": F.leaky_relu(y, 0.2)}[act])
        return torch.stack(ys)
    return _GBatchNormAct.apply(_act(x), gamma, beta, running_mean, running_var, stats, training, momentum, eps,
                                act)


# ------------------------------------------------------------------------------------ loss
class _GBCE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target):
        G, N, ld = logits.shape
        loss, dl = Fn.bce_logits(logits.reshape(G * N, ld), target, scale=1.0 / N)
        ctx.save_for_backward(dl)
        ctx.shape = logits.shape
        return (loss / N).reshape(())

    @staticmethod
    def backward(ctx, g):
        (dl,) = ctx.saved_tensors
        return (dl.float() * g).to(dl.dtype).view(ctx.shape), None


def bce_with_logits(logits, target):
    """SUM over the groups of each group's mean BCE-with-logits on column 0 of logits [G, N, ld]:
    every client's logit gradient is exactly its own mean-loss gradient."""
    G = logits.shape[0]
    if not logits.is_cuda:
        return sum(F.binary_cross_entropy_with_logits(logits[g, :, 0].float(),
                                                      torch.full((logits.shape[1],), float(target)))
                   for g in range(G))
    return _GBCE.apply(_act(logits), target)
