"""Autograd ops for the tabular nets on the HIP kernels of csrc/kernels/tabular.hip (exact fp32).

Device tensors run the fused kernels (linear + bias + activation on fp32 MFMA, BatchNorm1d +
activation, soft-target CE, MSE+KL, Philox reparameterisation); CPU tensors run the identical
PyTorch composition, so the models are written once (``models/tabular.py``).
"""
from __future__ import annotations

import ctypes
import itertools

import torch
import torch.nn.functional as F

from . import _lib
from ._lib import check, ptr, stream

vp, i32, i64, f32, u64 = _lib.vp, _lib.i32, _lib.i64, _lib.f32, _lib.u64
ACT = {"none": 0, "relu": 1, "leaky_relu": 2}


class GemmF32Args(ctypes.Structure):
    _fields_ = [("A", vp), ("B", vp), ("C", vp), ("bias", vp),
                ("sam", i64), ("sak", i64), ("sbk", i64), ("sbn", i64), ("ldc", i64),
                ("M", i32), ("N", i32), ("K", i32), ("act", i32), ("accumulate", i32),
                ("reserved", i32), ("slope", f32), ("alpha", f32)]


_lib.register_signatures({
    "ddl_gemm_f32": [ctypes.POINTER(GemmF32Args), vp],
    "ddl_bias_act_bwd": [vp, vp, vp, vp, i32, i32, i32, f32, vp],
    "ddl_bn1d_fwd": [vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, f32, f32, i32, f32, vp],
    "ddl_bn1d_bwd": [vp, vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, f32, i32, vp],
    "ddl_ce_f32": [vp, vp, vp, i32, i32, vp, vp, vp],
    "ddl_reparam": [vp, vp, vp, vp, i64, u64, u64, vp],
})


def K():
    k = _lib.kernels()
    assert k.ddl_gemm_f32_args_size() == ctypes.sizeof(GemmF32Args), "GemmF32Args ABI mismatch"
    return k


def gemm_f32(A, B, C, M, N, Kd, sam, sak, sbk, sbn, bias=None, act=0, slope=0.01,
             accumulate=False, alpha=1.0):
    a = GemmF32Args()
    a.A, a.B, a.C, a.bias = ptr(A), ptr(B), ptr(C), ptr(bias)
    a.sam, a.sak, a.sbk, a.sbn, a.ldc = sam, sak, sbk, sbn, C.stride(0)
    a.M, a.N, a.K, a.act, a.accumulate = M, N, Kd, act, int(accumulate)
    a.slope, a.alpha = slope, alpha
    check(K().ddl_gemm_f32(ctypes.byref(a), stream()), "gemm_f32")
    return C


def _act_torch(y, act, slope):
    return F.relu(y) if act == 1 else (F.leaky_relu(y, slope) if act == 2 else y)


# ----------------------------------------------------------------------------------- linear
class _LinearAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, act, slope):
        x2 = x.reshape(-1, x.shape[-1]).contiguous()
        M, Kd = x2.shape
        N = w.shape[0]
        wc = w.contiguous()
        y = torch.empty(M, N, dtype=torch.float32, device=x.device)
        gemm_f32(x2, wc, y, M, N, Kd, Kd, 1, 1, Kd, bias=b, act=act, slope=slope)
        ctx.save_for_backward(x2, wc, y if act else None)
        ctx.act, ctx.slope, ctx.has_b, ctx.shape = act, slope, b is not None, x.shape
        return y.view(*x.shape[:-1], N)

    @staticmethod
    def backward(ctx, dy):
        x2, w, y = ctx.saved_tensors
        M, Kd = x2.shape
        N = w.shape[0]
        d = dy.reshape(M, N).contiguous().float()
        db = torch.zeros(N, dtype=torch.float32, device=d.device) if ctx.has_b else None
        if ctx.act or db is not None:
            dz = torch.empty_like(d) if ctx.act else d
            check(K().ddl_bias_act_bwd(ptr(d), ptr(y), ptr(dz) if ctx.act else None, ptr(db), M, N,
                                       ctx.act, ctx.slope, stream()), "bias_act_bwd")
            d = dz
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty(M, Kd, dtype=torch.float32, device=d.device)
            gemm_f32(d, w, dx, M, Kd, N, N, 1, Kd, 1)                 # dX = dZ W
            dx = dx.view(ctx.shape)
        if ctx.needs_input_grad[1]:
            dw = torch.empty(N, Kd, dtype=torch.float32, device=d.device)
            gemm_f32(d, x2, dw, N, Kd, M, 1, N, Kd, 1)                # dW = dZ^T X
        return dx, dw, db, None, None


def linear_act(x, w, b=None, act="none", slope=0.01):
    """y = act(x @ w.T + b) — one fused fp32-MFMA kernel on the device."""
    code = ACT[act] if isinstance(act, str) else int(act)
    if not x.is_cuda:
        return _act_torch(F.linear(x, w, b), code, slope)
    return _LinearAct.apply(x.float(), w, b, code, slope)


# ------------------------------------------------------------------------------ BatchNorm1d
class _BN1dAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, rm, rv, training, momentum, eps, act, slope):
        x2 = x.contiguous().float()
        M, C = x2.shape
        y = torch.empty_like(x2)
        mean = torch.empty(C, dtype=torch.float32, device=x.device)
        rstd = torch.empty_like(mean)
        check(K().ddl_bn1d_fwd(ptr(x2), ptr(gamma), ptr(beta), ptr(rm), ptr(rv), ptr(y), ptr(mean),
                               ptr(rstd), M, C, int(training), float(momentum), float(eps), act,
                               float(slope), stream()), "bn1d_fwd")
        ctx.save_for_backward(x2, y, mean, rstd, gamma)
        ctx.act, ctx.slope, ctx.training = act, slope, int(bool(training))
        return y

    @staticmethod
    def backward(ctx, dy):
        x2, y, mean, rstd, gamma = ctx.saved_tensors
        M, C = x2.shape
        dx = torch.empty_like(x2)
        dg = torch.zeros(C, dtype=torch.float32, device=x2.device)
        db = torch.zeros_like(dg)
        check(K().ddl_bn1d_bwd(ptr(dy.contiguous().float()), ptr(y), ptr(x2), ptr(mean), ptr(rstd),
                               ptr(gamma), ptr(dx), ptr(dg), ptr(db), M, C, ctx.act, ctx.slope,
                               ctx.training, stream()), "bn1d_bwd")
        return dx, dg, db, None, None, None, None, None, None, None


def batch_norm1d_act(x, gamma, beta, running_mean, running_var, training, momentum=0.1, eps=1e-5,
                     act="none", slope=0.01):
    code = ACT[act] if isinstance(act, str) else int(act)
    if not x.is_cuda:
        y = F.batch_norm(x, running_mean, running_var, gamma, beta, training, momentum, eps)
        return _act_torch(y, code, slope)
    # eval mode runs the same native kernels with the running statistics (fixed affine backward)
    return _BN1dAct.apply(x, gamma, beta, running_mean, running_var, training, momentum, eps,
                          code, slope)


# ------------------------------------------------------------------------------------ losses
class _CE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target):
        lg = logits.contiguous().float()
        M, C = lg.shape
        loss = torch.zeros(1, dtype=torch.float32, device=lg.device)
        dl = torch.empty_like(lg)
        soft = target.dtype.is_floating_point
        t = target.contiguous().float() if soft else target.contiguous().int()
        check(K().ddl_ce_f32(ptr(lg), ptr(t) if soft else None, None if soft else ptr(t), M, C,
                             ptr(loss), ptr(dl), stream()), "ce_f32")
        ctx.save_for_backward(dl)
        return loss.reshape(())

    @staticmethod
    def backward(ctx, g):
        (dl,) = ctx.saved_tensors
        return dl * g, None


def cross_entropy(logits, target):
    """nn.CrossEntropyLoss (mean) with hard labels or probability targets (vfl.py:51,79)."""
    if not logits.is_cuda:
        return F.cross_entropy(logits, target)
    return _CE.apply(logits, target)


class _MSEKL(torch.autograd.Function):
    @staticmethod
    def forward(ctx, xr, x, mu, lv):
        xr_, x_, mu_, lv_ = (t.contiguous().float() for t in (xr, x, mu, lv))
        loss = torch.zeros(1, dtype=torch.float32, device=xr.device)
        dxr, dmu, dlv = torch.empty_like(xr_), torch.empty_like(mu_), torch.empty_like(lv_)
        check(K().ddl_mse_kl(ptr(xr_), ptr(x_), xr_.numel(), ptr(mu_), ptr(lv_), mu_.numel(), 1.0,
                             1.0, ptr(loss), ptr(dxr), ptr(dmu), ptr(dlv), stream()), "mse_kl")
        ctx.save_for_backward(dxr, dmu, dlv)
        return loss.reshape(())

    @staticmethod
    def backward(ctx, g):
        dxr, dmu, dlv = ctx.saved_tensors
        return dxr * g, None, dmu * g, dlv * g


def mse_kl(xr, x, mu, logvar):
    """customLoss: MSE(sum) + KL(N(mu, sigma) || N(0, 1)) — one fused reduction on the device."""
    if not xr.is_cuda:
        return F.mse_loss(xr, x, reduction="sum") - 0.5 * torch.sum(1 + logvar - mu.pow(2) - logvar.exp())
    return _MSEKL.apply(xr, x, mu, logvar)


_REPARAM_CTR = itertools.count()


class _Reparam(torch.autograd.Function):
    @staticmethod
    def forward(ctx, mu, lv, seed):
        m, l = mu.contiguous().float(), lv.contiguous().float()
        eps, z = torch.empty_like(m), torch.empty_like(m)
        check(K().ddl_reparam(ptr(m), ptr(l), ptr(eps), ptr(z), m.numel(), seed,
                              next(_REPARAM_CTR) * (1 << 32), stream()), "reparam")
        ctx.save_for_backward(eps, l)
        return z

    @staticmethod
    def backward(ctx, dz):
        eps, l = ctx.saved_tensors
        return dz, dz * eps * 0.5 * torch.exp(0.5 * l), None


def reparameterize(mu, logvar, seed=None):
    """z = mu + eps * exp(logvar / 2): device draws eps with Philox (seed from torch's RNG)."""
    if not mu.is_cuda:
        return mu + torch.randn_like(mu) * torch.exp(0.5 * logvar)
    if seed is None:
        seed = int(torch.randint(0, 2 ** 62, (1,)).item())
    return _Reparam.apply(mu, logvar, seed)
