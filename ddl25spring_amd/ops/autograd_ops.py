"""Autograd-composable ops for ``torch.nn.Module`` models (LLaMA stages, tabular nets, GANs).

On device tensors every op below is a HIP kernel (MFMA implicit-GEMM for the linears, the fused
LLaMA kernels of csrc/kernels/llama.hip, fused CE over the vocabulary). The activation dtype picks
the precision: bf16 activations run the bf16-MFMA kernels (parameters stay fp32 ``nn.Parameter``,
cast to a bf16 shadow per forward); fp32 activations (the reference's precision) run
ops/llama_f32.py (csrc/kernels/llama_f32.hip + the fp32 conv engine). Weight gradients are fp32. On CPU tensors the same functions run plain PyTorch fp32 ops, so module code is written once
and is testable without a GPU.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from . import _lib
from . import functional as Fn
from . import llama_f32 as L32
from ._lib import check, ptr, stream

vp, i32, i64, f32 = _lib.vp, _lib.i32, _lib.i64, _lib.f32
_lib.register_signatures({
    "ddl_embedding_fwd": [vp, vp, vp, i32, i32, vp],
    "ddl_embedding_bwd": [vp, vp, vp, i32, i32, i32, vp],
    "ddl_rmsnorm_fwd": [vp, vp, vp, vp, i32, i32, f32, vp],
    "ddl_rmsnorm_bwd": [vp, vp, vp, vp, vp, vp, vp, i32, i32, vp],
    "ddl_rmsnorm_bwd_set_rows": [i32],
    "ddl_swiglu_fwd": [vp, vp, i32, i32, vp],
    "ddl_swiglu_bwd": [vp, vp, vp, i32, i32, vp],
    "ddl_add": [vp, vp, vp, i64, vp],
    "ddl_attn_fwd": [vp, vp, vp, vp, vp, i32, i32, i32, i32, f32, vp],
    "ddl_attn_bwd": [vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, f32, vp],
    "ddl_ce_vocab_lse": [vp, vp, i32, i32, i32, vp, i32, vp, vp, vp],
    "ddl_ce_vocab_grad": [vp, vp, i32, i32, i32, vp, vp, vp, i32, vp, vp],
    "ddl_ce_vocab_fused": [vp, vp, i32, i32, i32, vp, i32, vp, vp, vp],
    "ddl_ce_vocab_scale": [vp, i64, vp, vp],
})


def K():
    return _lib.kernels()


def _bf16_weight(w: torch.Tensor) -> torch.Tensor:
    sh = getattr(w, "_ddl_bf16", None)  # FlatAdam(bf16_shadow=True) keeps it current: no cast
    if sh is not None:
        return sh
    return Fn.to_bf16(w.detach().contiguous())


def _grad_sink(p: torch.Tensor):
    """``p.grad`` itself when the parameter's optimizer lets backward accumulate into it in place
    (``FlatAdam(fused=True)`` marks its parameters), else None and autograd accumulates. Saves the
    zero-fill of a fresh gradient and AccumulateGrad's add pass (37 MB each for the 32k x 288
    embedding / LM head, per micro-batch)."""
    if not getattr(p, "_ddl_fuse_grad", False):
        return None
    g = p.grad
    if g is None or g.dtype != torch.float32 or not g.is_contiguous() or g.device != p.device:
        return None
    return g


def _grad_ready(p: torch.Tensor) -> None:
    """A fused accumulation bypasses AccumulateGrad, so run what its post-accumulate hook would:
    the DP bucketer registers its hook as ``p._ddl_on_grad``."""
    cb = getattr(p, "_ddl_on_grad", None)
    if cb is not None:
        cb(p)


# ------------------------------------------------------------------------------------- linear
# A plain (no bias / residual epilogue) linear with a vocabulary-sized output runs its forward on
# the dedicated wide-output GEMM (csrc/kernels/gemm_bf16.hip): on the LLaMA-288 LM head
# (8192 x 288 -> 32000) the MFMA conv-GEMM takes 389 us (its 9-step reduction leaves the 524 MB
# bf16 output write exposed) and hipBLASLt 264 us (scripts/gemm_vs_blas.py,
# profiles/gemm_vs_blas_r2f.txt); every block-sized linear, and the LM head's backward, run on
# the conv-GEMM.
WIDE_FWD_MIN_OUT = 8192


class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, residual):
        C = x.shape[-1]
        Kout = w.shape[0]
        x2 = x.reshape(-1, C).contiguous()
        T = x2.shape[0]
        geom = Fn.ConvGeom(1, T, 1, 1, C, Kout, 1, 1, 1, 0)
        wb = _bf16_weight(w).view(1, Kout, 1, 1, C)
        res = residual.reshape(1, T, 1, 1, Kout).contiguous() if residual is not None else None
        if b is None and res is None and Kout >= WIDE_FWD_MIN_OUT and Fn.gemm_nt_ok(C, Kout):
            y = Fn.gemm_nt_bf16(x2, wb.view(Kout, C))
        else:
            y = Fn.conv_fwd(x2.view(1, T, 1, 1, C), wb, geom,
                            bias=None if b is None else b.detach().view(1, Kout), residual=res)
        ctx.save_for_backward(x2, wb)
        ctx.geom, ctx.has_b, ctx.has_res, ctx.xshape = geom, b is not None, residual is not None, x.shape
        ctx.w = w
        return y.view(*x.shape[:-1], Kout)

    @staticmethod
    def backward(ctx, dy):
        x2, wb = ctx.saved_tensors
        g = ctx.geom
        dy5 = dy.reshape(1, g.N, 1, 1, g.K).to(torch.bfloat16).contiguous()
        dx = dw = db = None
        if ctx.needs_input_grad[1]:
            sink = _grad_sink(ctx.w)
            # accumulate straight into the parameter's grad when it has a flat-buffer sink
            dwt = sink.view(1, g.K, 1, 1, g.C) if sink is not None else \
                torch.zeros(1, g.K, 1, 1, g.C, dtype=torch.float32, device=dy.device)
            # dX and dW read the same dY: one (possibly paired) launch
            dx = Fn.conv_dgrad_wgrad(dy5, wb, x2.view(1, g.N, 1, 1, g.C), g, dwt,
                                     want_dx=ctx.needs_input_grad[0])
            if dx is not None:
                dx = dx.view(ctx.xshape)
            if sink is not None:
                _grad_ready(ctx.w)
            else:
                dw = dwt.view(g.K, g.C)
        elif ctx.needs_input_grad[0]:
            dx = Fn.conv_dgrad(dy5, wb, g).view(ctx.xshape)
        if ctx.has_b and ctx.needs_input_grad[2]:
            db = torch.zeros(1, g.K, dtype=torch.float32, device=dy.device)
            Fn.channel_sum(dy5.view(1, g.N, g.K), db)
            db = db.view(g.K)
        dres = dy if ctx.has_res else None
        return dx, dw, db, dres


def _f32(x) -> bool:
    """fp32 device activations take the reference-precision kernels (ops/llama_f32.py)."""
    return x.dtype == torch.float32


def linear(x, w, b=None, residual=None):
    """y = x @ w.T (+ b) (+ residual). Device: one MFMA GEMM with the bias / residual in its epilogue
    (bf16 activations: bf16 MFMA; fp32 activations: the X6 / exact-fp32 conv engine)."""
    if not x.is_cuda:
        y = F.linear(x, w, b)
        return y + residual if residual is not None else y
    if _f32(x):
        return L32.LinearF32.apply(x, w, b, None if residual is None else residual.float())
    if x.dtype != torch.bfloat16:
        x = x.to(torch.bfloat16)
    if residual is not None and residual.dtype != torch.bfloat16:
        residual = residual.to(torch.bfloat16)
    return _Linear.apply(x, w, b, residual)


# ------------------------------------------------------------------------------------ rmsnorm
class _RMSNorm(torch.autograd.Function):
    """y = x * rsqrt(mean(x^2) + eps) * g. With ``fork`` the function also returns x itself (a view)
    for a pre-norm block's residual branch, so the two gradients of x arrive in one backward call
    and the residual one is added inside the RMSNorm backward kernel instead of by a separate
    autograd gradient-sum pass."""

    @staticmethod
    def forward(ctx, x, g, eps, fork):
        D = x.shape[-1]
        x2 = x.reshape(-1, D).contiguous()
        T = x2.shape[0]
        y = torch.empty_like(x2)
        rstd = torch.empty(T, dtype=torch.float32, device=x.device)
        gd = g.detach().float().contiguous()
        check(K().ddl_rmsnorm_fwd(ptr(x2), ptr(gd), ptr(y), ptr(rstd), T, D, float(eps), stream()),
              "rmsnorm_fwd")
        ctx.save_for_backward(x2, gd, rstd)
        ctx.shape, ctx.g = x.shape, g
        if fork:
            return y.view(x.shape), x.view_as(x)
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, dy, dres=None):
        x2, gd, rstd = ctx.saved_tensors
        T, D = x2.shape
        dx = torch.empty_like(x2)
        sink = _grad_sink(ctx.g) if ctx.needs_input_grad[1] else None
        dg = sink if sink is not None else torch.zeros(D, dtype=torch.float32, device=x2.device)
        if dy is None:
            dy = torch.zeros_like(x2)
        dyc = dy.reshape(T, D).to(torch.bfloat16).contiguous()
        drc = None if dres is None else dres.reshape(T, D).to(torch.bfloat16).contiguous()
        check(K().ddl_rmsnorm_bwd(ptr(x2), ptr(gd), ptr(rstd), ptr(dyc), ptr(drc), ptr(dx), ptr(dg),
                                  T, D, stream()), "rmsnorm_bwd")
        if sink is not None:
            _grad_ready(ctx.g)
            dg = None
        return dx.view(ctx.shape), dg, None, None


def rmsnorm(x, g, eps=1e-6):
    if not x.is_cuda:
        return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps) * g
    if _f32(x):
        return L32.RMSNormF32.apply(x, g, eps, False)
    return _RMSNorm.apply(x.to(torch.bfloat16), g, eps, False)


def rmsnorm_fork(x, g, eps=1e-6):
    """(rmsnorm(x, g), x) for a pre-norm residual block; on the GPU the residual branch's gradient
    is summed into dx by the RMSNorm backward kernel."""
    if not x.is_cuda:
        return rmsnorm(x, g, eps), x
    if _f32(x):
        return L32.RMSNormF32.apply(x, g, eps, True)
    return _RMSNorm.apply(x.to(torch.bfloat16), g, eps, True)


# ------------------------------------------------------------------------------------- swiglu
class _SwiGLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ab):
        F2 = ab.shape[-1]
        ab2 = ab.reshape(-1, F2).contiguous()
        T = ab2.shape[0]
        h = torch.empty(T, F2 // 2, dtype=torch.bfloat16, device=ab.device)
        check(K().ddl_swiglu_fwd(ptr(ab2), ptr(h), T, F2 // 2, stream()), "swiglu_fwd")
        ctx.save_for_backward(ab2)
        ctx.shape = ab.shape
        return h.view(*ab.shape[:-1], F2 // 2)

    @staticmethod
    def backward(ctx, dh):
        (ab2,) = ctx.saved_tensors
        T, F2 = ab2.shape
        dab = torch.empty_like(ab2)
        dhc = dh.reshape(T, F2 // 2).to(torch.bfloat16).contiguous()
        check(K().ddl_swiglu_bwd(ptr(ab2), ptr(dhc), ptr(dab), T, F2 // 2, stream()), "swiglu_bwd")
        return dab.view(ctx.shape)


def swiglu(ab):
    """silu(a) * b for ab = [a | b] along the last dim."""
    if not ab.is_cuda:
        a, b = ab.chunk(2, -1)
        return F.silu(a) * b
    if _f32(ab):
        return L32.SwiGLUF32.apply(ab)
    return _SwiGLU.apply(ab.to(torch.bfloat16))


# ---------------------------------------------------------------------------------- embedding
class _Embedding(torch.autograd.Function):
    @staticmethod
    def forward(ctx, idx, w, pad_idx):
        idx32 = idx.to(torch.int32).contiguous().reshape(-1)
        T, D = idx32.numel(), w.shape[1]
        y = torch.empty(T, D, dtype=torch.bfloat16, device=w.device)
        wd = w.detach().float().contiguous()
        check(K().ddl_embedding_fwd(ptr(idx32), ptr(wd), ptr(y), T, D, stream()), "embedding_fwd")
        ctx.save_for_backward(idx32)
        ctx.wshape, ctx.pad, ctx.ishape, ctx.w = w.shape, pad_idx, idx.shape, w
        return y.view(*idx.shape, D)

    @staticmethod
    def backward(ctx, dy):
        (idx32,) = ctx.saved_tensors
        V, D = ctx.wshape
        sink = _grad_sink(ctx.w) if ctx.needs_input_grad[1] else None
        dw = sink if sink is not None else torch.zeros(V, D, dtype=torch.float32, device=dy.device)
        dyc = dy.reshape(-1, D).to(torch.bfloat16).contiguous()
        check(K().ddl_embedding_bwd(ptr(idx32), ptr(dyc), ptr(dw), idx32.numel(), D,
                                    -1 if ctx.pad is None else int(ctx.pad), stream()),
              "embedding_bwd")
        if sink is not None:
            _grad_ready(ctx.w)
            dw = None
        return None, dw, None


def embedding(idx, w, padding_idx=None, dtype=None):
    """Row gather; on the device the output dtype is ``dtype`` (default bf16): float32 selects the
    reference-precision path for everything downstream."""
    if not w.is_cuda:
        return F.embedding(idx, w, padding_idx)
    if dtype == torch.float32:
        return L32.EmbeddingF32.apply(idx, w, padding_idx)
    return _Embedding.apply(idx, w, padding_idx)


def add(a, b):
    if not a.is_cuda:
        return a + b
    return _Add.apply(a.to(torch.bfloat16), b.to(torch.bfloat16))


class _Add(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b):
        ac, bc = a.contiguous(), b.contiguous()
        y = torch.empty_like(ac)
        check(K().ddl_add(ptr(ac), ptr(bc), ptr(y), ac.numel(), stream()), "add")
        return y

    @staticmethod
    def backward(ctx, dy):
        return dy, dy


# ---------------------------------------------------------------------------------- attention
_ROPE: dict = {}


def rope_tables(S, hd, device, base=10000.0):
    key = (S, hd, str(device), base)
    t = _ROPE.get(key)
    if t is None:
        inv = base ** (-torch.arange(0, hd, 2, dtype=torch.float64) / hd)
        ang = torch.arange(S, dtype=torch.float64)[:, None] * inv[None]
        t = (torch.cos(ang).float().to(device).contiguous(), torch.sin(ang).float().to(device).contiguous())
        _ROPE[key] = t
    return t


def apply_rope_ref(x, cos, sin):
    """x [..., S, H, hd] with interleaved pairs (2i, 2i+1)."""
    x0, x1 = x[..., 0::2], x[..., 1::2]
    c = cos[:, None, :]
    s = sin[:, None, :]
    out = torch.empty_like(x)
    out[..., 0::2] = x0 * c - x1 * s
    out[..., 1::2] = x0 * s + x1 * c
    return out


def attention_ref(qkv, H, hd):
    B, S, _ = qkv.shape
    q, k, v = qkv.view(B, S, 3, H, hd).unbind(2)
    cos, sin = rope_tables(S, hd, qkv.device)
    q, k = apply_rope_ref(q, cos, sin), apply_rope_ref(k, cos, sin)
    o = F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2),
                                       is_causal=True)
    return o.transpose(1, 2).reshape(B, S, H * hd)


class _Attention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, H, hd):
        B, S, _ = qkv.shape
        qc = qkv.contiguous()
        cos, sin = rope_tables(S, hd, qkv.device)
        o = torch.empty(B, S, H * hd, dtype=torch.bfloat16, device=qkv.device)
        lse = torch.empty(B, H, S, dtype=torch.float32, device=qkv.device)
        scale = 1.0 / math.sqrt(hd)
        check(K().ddl_attn_fwd(ptr(qc), ptr(o), ptr(lse), ptr(cos), ptr(sin), B, S, H, hd, scale,
                               stream()), "attn_fwd")
        ctx.save_for_backward(qc, o, lse)
        ctx.H, ctx.hd, ctx.scale = H, hd, scale
        return o

    @staticmethod
    def backward(ctx, do):
        qc, o, lse = ctx.saved_tensors
        B, S, _ = qc.shape
        cos, sin = rope_tables(S, ctx.hd, qc.device)
        dqkv = torch.empty_like(qc)
        delta = torch.empty_like(lse)
        doc = do.to(torch.bfloat16).contiguous()
        check(K().ddl_attn_bwd(ptr(qc), ptr(o), ptr(doc), ptr(lse), ptr(delta), ptr(dqkv), ptr(cos),
                               ptr(sin), B, S, ctx.H, ctx.hd, ctx.scale, stream()), "attn_bwd")
        return dqkv, None, None


def causal_attention(qkv, n_heads, head_dim):
    """Causal multi-head attention with RoPE on q, k. qkv: [B, S, 3*H*hd] -> [B, S, H*hd]."""
    if not qkv.is_cuda:
        return attention_ref(qkv, n_heads, head_dim)
    if _f32(qkv):
        return L32.AttentionF32.apply(qkv, n_heads, head_dim)
    return _Attention.apply(qkv.to(torch.bfloat16), n_heads, head_dim)


# ------------------------------------------------------------------------------- LM loss
CE_FUSED_MAX_V = 32768  # == CE_RC * 256 * 8 in loss.hip


class _VocabCE(torch.autograd.Function):
    """Mean token CE over the rows of bf16 logits [..., V] with int32 labels. No host sync (the
    1/#valid normaliser is a device scalar). The forward makes the loss and the gradient at unit
    upstream scale from one read of the logits (``ddl_ce_vocab_fused``, V <= 32768; wider
    vocabularies take the lse-then-gradient pair); the backward rescales that
    gradient in place by the upstream gradient only when it is not 1 (checked on the device). A
    second backward through the same graph recomputes the gradient first."""

    @staticmethod
    def forward(ctx, logits, labels, ignore_index, scale):
        V = logits.shape[-1]
        lg = logits.reshape(-1, V)
        if not lg.is_contiguous():
            lg = lg.contiguous()
        R = lg.shape[0]
        lab = labels.reshape(-1)
        inv = (lab != ignore_index).sum(dtype=torch.float32).clamp_min_(1.0).reciprocal_().reshape(1)
        if scale != 1.0:
            inv.mul_(scale)
        loss = torch.zeros(1, dtype=torch.float32, device=lg.device)
        # the fused loss + gradient pass writes a [R, V] gradient: only worth it when one is needed
        # (no_grad / eval forwards keep just the per-row log-sum-exp)
        if V > CE_FUSED_MAX_V or not ctx.needs_input_grad[0]:
            lse = torch.empty(R, dtype=torch.float32, device=lg.device)
            check(K().ddl_ce_vocab_lse(ptr(lg), ptr(lab), R, V, V, ptr(inv), int(ignore_index), ptr(loss),
                                       ptr(lse), stream()), "ce_vocab_lse")
            d = None
            ctx.lse = lse
        else:
            d = torch.empty_like(lg)
            check(K().ddl_ce_vocab_fused(ptr(lg), ptr(lab), R, V, V, ptr(inv), int(ignore_index),
                                         ptr(loss), ptr(d), stream()), "ce_vocab_fused")
        ctx.save_for_backward(lg, lab, inv, d)
        ctx.shape, ctx.ignore, ctx.used = logits.shape, int(ignore_index), False
        return loss[0]

    @staticmethod
    def backward(ctx, g):
        lg, lab, inv, d = ctx.saved_tensors
        R, V = lg.shape
        if d is None:  # wide vocabulary: the gradient from the saved log-sum-exp, scaled by g
            gg = g.detach().to(torch.float32).reshape(1).contiguous()
            d = torch.empty_like(lg)
            check(K().ddl_ce_vocab_grad(ptr(lg), ptr(lab), R, V, V, ptr(ctx.lse), ptr(inv), ptr(gg),
                                        ctx.ignore, ptr(d), stream()), "ce_vocab_grad")
            return d.view(ctx.shape), None, None, None
        if ctx.used:  # the unit-scale gradient was already rescaled by an earlier backward
            d = torch.empty_like(lg)
            junk = torch.zeros(1, dtype=torch.float32, device=lg.device)
            check(K().ddl_ce_vocab_fused(ptr(lg), ptr(lab), R, V, V, ptr(inv), ctx.ignore, ptr(junk),
                                         ptr(d), stream()), "ce_vocab_fused")
        ctx.used = True
        gg = g.detach().to(torch.float32).reshape(1).contiguous()
        check(K().ddl_ce_vocab_scale(ptr(d), d.numel(), ptr(gg), stream()), "ce_vocab_scale")
        return d.view(ctx.shape), None, None, None


def cross_entropy_vocab(logits, targets, ignore_index=-100, scale: float = 1.0):
    """``scale`` x mean token cross-entropy; one fused kernel computes loss and d(logits).
    Pass a constant factor (e.g. 1 / micro-batches) as ``scale`` rather than multiplying the
    returned loss: the gradient is then final in the forward pass and the backward has no
    rescaling pass over the [rows, V] gradient."""
    if not logits.is_cuda:
        lg = logits.reshape(-1, logits.shape[-1])
        if lg.dtype not in (torch.float32, torch.float64):
            lg = lg.float()
        return scale * F.cross_entropy(lg, targets.reshape(-1).long(), ignore_index=ignore_index)
    if _f32(logits):
        return L32.VocabCEF32.apply(logits, targets.to(torch.int32).contiguous(), ignore_index, float(scale))
    if logits.dtype != torch.bfloat16:
        logits = logits.to(torch.bfloat16)
    return _VocabCE.apply(logits, targets.to(torch.int32).contiguous(), ignore_index, float(scale))


# ===================================================================== image ops (NHWC, GANs)
# Activations are NHWC [N, H, W, C]; conv weights are fp32 parameters in the kernels' layout
# [K, R, S, C] (conv) / [Cin, R, S, Cout] (transposed conv). Channel counts must be multiples of
# 32 on the device (pad small ones, e.g. RGB 3 -> 32, with zero weights: they stay exactly zero).
# Precision follows the activation dtype: fp32 device activations (the DCGAN's default, the
# reference's precision) run the fp32 kernels (conv_f32.hip / bn_f32.hip / fp32 BCE) with the fp32
# parameters themselves as operands; anything else runs bf16 on the bf16 weight shadow.
def _geom(x_shape, C, K, R, S, stride, pad):
    N, H, W = x_shape[0], x_shape[1], x_shape[2]
    return Fn.ConvGeom(1, N, H, W, C, K, R, S, stride, pad)


def _img_act(x):
    return x if x.dtype in (torch.float32, torch.bfloat16) else x.to(torch.bfloat16)


def _img_weight(w, dtype):
    return w.detach().contiguous() if dtype == torch.float32 else _bf16_weight(w)


class _Conv2d(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, stride, pad, want_stats):
        Kc, R, S, C = w.shape
        g = _geom(x.shape, C, Kc, R, S, stride, pad)
        wb = _img_weight(w, x.dtype).view(1, Kc, R, S, C)
        x = x.contiguous()
        stats = Fn.stats_buffer(1, Kc, x.device, like=x) if want_stats else None
        y = Fn.conv_fwd(x.view(1, *x.shape), wb, g, stats=stats)
        ctx.save_for_backward(x, wb)
        ctx.g = g
        if want_stats and torch.is_tensor(stats):
            ctx.mark_non_differentiable(stats)
        return y.view(g.N, g.P, g.Q, Kc), stats

    @staticmethod
    def backward(ctx, dy, _dstats):
        x, wb = ctx.saved_tensors
        g = ctx.g
        dy5 = dy.to(x.dtype).contiguous().view(1, g.N, g.P, g.Q, g.K)
        dx = dw = None
        if ctx.needs_input_grad[1]:
            dw = torch.zeros(1, g.K, g.R, g.S, g.C, dtype=torch.float32, device=dy.device)
            dx = Fn.conv_dgrad_wgrad(dy5, wb, x.contiguous().view(1, *x.shape), g, dw,
                                     want_dx=ctx.needs_input_grad[0])
            dx = None if dx is None else dx.view(x.shape)
            dw = dw.view(g.K, g.R, g.S, g.C)
        elif ctx.needs_input_grad[0]:
            dx = Fn.conv_dgrad(dy5, wb, g).view(x.shape)
        return dx, dw, None, None, None


def conv2d(x, w, stride=1, pad=0, with_stats=False):
    """NHWC conv, weight [K, R, S, C]. with_stats: also return the per-channel (sum, sumsq) [1,2,K]
    of the output, computed in the MFMA epilogue (feeds ``batch_norm_act``)."""
    if not x.is_cuda:
        y = F.conv2d(x.permute(0, 3, 1, 2), w.permute(0, 3, 1, 2), stride=stride, padding=pad)
        y = y.permute(0, 2, 3, 1)
        return (y, None) if with_stats else y
    y, st = _Conv2d.apply(_img_act(x), w, stride, pad, with_stats)
    return (y, st) if with_stats else y


class _ConvT2d(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, stride, pad):
        Cin, R, S, Cout = w.shape
        N, Hi, Wi, _ = x.shape
        Ho, Wo = (Hi - 1) * stride - 2 * pad + R, (Wi - 1) * stride - 2 * pad + S
        g = Fn.ConvGeom(1, N, Ho, Wo, Cout, Cin, R, S, stride, pad)  # the conv this one transposes
        assert (g.P, g.Q) == (Hi, Wi), "transposed conv geometry must invert exactly"
        wb = _img_weight(w, x.dtype).view(1, Cin, R, S, Cout)
        y = Fn.conv_dgrad(x.contiguous().view(1, N, Hi, Wi, Cin), wb, g)
        ctx.save_for_backward(x, wb)
        ctx.g = g
        return y.view(N, Ho, Wo, Cout)

    @staticmethod
    def backward(ctx, dy):
        x, wb = ctx.saved_tensors
        g = ctx.g
        dy5 = dy.to(x.dtype).contiguous().view(1, g.N, g.H, g.W, g.C)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = Fn.conv_fwd(dy5, wb, g).view(x.shape)
        if ctx.needs_input_grad[1]:
            dw = torch.zeros(1, g.K, g.R, g.S, g.C, dtype=torch.float32, device=dy.device)
            Fn.conv_wgrad(x.contiguous().view(1, *x.shape), dy5, g, dw)
            dw = dw.view(g.K, g.R, g.S, g.C)
        return dx, dw, None, None


def conv_transpose2d(x, w, stride=1, pad=0):
    """NHWC transposed conv (nn.ConvTranspose2d, no bias), weight [Cin, R, S, Cout]: runs as the
    dgrad of the conv it transposes (phase-decomposed for stride 2), backward = conv fwd + wgrad."""
    if not x.is_cuda:
        y = F.conv_transpose2d(x.permute(0, 3, 1, 2), w.permute(0, 3, 1, 2), stride=stride, padding=pad)
        return y.permute(0, 2, 3, 1)
    return _ConvT2d.apply(_img_act(x), w, stride, pad)


_BN_ACT = {"none": 0, "relu": 1, "leaky_relu": 3}  # bn_apply codes (3 = leaky 0.2)


class _BatchNormAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, running_mean, running_var, stats, training, momentum, eps, act):
        C = x.shape[-1]
        xg = x.contiguous().view(1, -1, C)
        M = xg.shape[1]
        if training and stats is None:
            stats = Fn.bn_stats(xg)
        if stats is None:
            stats = torch.zeros(1, 2, C, dtype=torch.float32, device=x.device)
        ga, be = gamma.detach().view(1, C), beta.detach().view(1, C)
        rm = running_mean.view(1, C) if running_mean is not None else None
        rv = running_var.view(1, C) if running_var is not None else None
        scale, shift, mean, rstd = Fn.bn_finalize(stats, ga, be, rm, rv, M, eps, momentum, training)
        y = Fn.bn_apply(xg, scale, shift, act=_BN_ACT[act])
        ctx.save_for_backward(xg, y, mean, rstd, ga)
        ctx.act, ctx.shape = act, x.shape
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, dy):
        xg, y, mean, rstd, ga = ctx.saved_tensors
        C = xg.shape[-1]
        d = dy.to(xg.dtype).contiguous().view_as(xg)
        ymask = None
        if ctx.act == "relu":
            ymask = y
        elif ctx.act == "leaky_relu":
            d = Fn.act_bwd(y, d, 2, 0.2)
        dgamma = torch.zeros(1, C, dtype=torch.float32, device=dy.device)
        dbeta = torch.zeros(1, C, dtype=torch.float32, device=dy.device)
        dx = Fn.bn_backward(d, ymask, xg, mean, rstd, ga, dgamma, dbeta)
        return dx.view(ctx.shape), dgamma.view(C), dbeta.view(C), None, None, None, None, None, None, None


def batch_norm_act(x, gamma, beta, running_mean=None, running_var=None, training=True,
                   momentum=0.1, eps=1e-5, act="none", stats=None):
    """BatchNorm over all but the last (channel) dim + fused activation ('none' | 'relu' |
    'leaky_relu' (slope 0.2)). ``stats`` (sum, sumsq) may come from a conv epilogue."""
    if not x.is_cuda:
        C = x.shape[-1]
        y = F.batch_norm(x.reshape(-1, C), running_mean, running_var, gamma, beta, training,
                         momentum, eps).view(x.shape)
        return {"none": y, "relu": F.relu(y), "leaky_relu": F.leaky_relu(y, 0.2)}[act]
    return _BatchNormAct.apply(_img_act(x), gamma, beta, running_mean, running_var, stats, training, momentum,
                               eps, act)


_ACT = {"relu": (1, 0.0), "leaky_relu": (2, 0.2), "tanh": (3, 0.0), "sigmoid": (4, 0.0)}


class _Act(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, kind):
        code, slope = _ACT[kind]
        y = Fn.act_fwd(x.contiguous(), code, slope)
        ctx.save_for_backward(y)
        ctx.code, ctx.slope = code, slope
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        return Fn.act_bwd(y, dy.to(y.dtype).contiguous(), ctx.code, ctx.slope), None


def activation(x, kind):
    """'relu' | 'leaky_relu' (0.2) | 'tanh' | 'sigmoid' — one elementwise HIP pass each way."""
    if not x.is_cuda:
        return {"relu": F.relu, "leaky_relu": lambda t: F.leaky_relu(t, 0.2),
                "tanh": torch.tanh, "sigmoid": torch.sigmoid}[kind](x)
    return _Act.apply(_img_act(x), kind)


class _BCE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target):
        R = logits.shape[0]
        loss, dl = Fn.bce_logits(logits.contiguous(), target, scale=1.0 / R)
        ctx.save_for_backward(dl)
        return (loss / R).reshape(())

    @staticmethod
    def backward(ctx, g):
        (dl,) = ctx.saved_tensors
        return (dl.float() * g).to(dl.dtype), None


def bce_with_logits(logits, target):
    """mean BCE-with-logits on column 0 of ``logits`` [R, ld] (the padded 1-unit head);
    target: python float (all rows) or fp32 [R]."""
    if not logits.is_cuda:
        t = target if torch.is_tensor(target) else torch.full((logits.shape[0],), float(target))
        return F.binary_cross_entropy_with_logits(logits[:, 0].float(), t.float())
    return _BCE.apply(_img_act(logits), target)
