"""Reference-precision (fp32) autograd ops of the LLaMA path (csrc/kernels/llama_f32.hip + the X6 /
exact-fp32 conv engine of conv_f32.hip for every linear).

The reference trains its LLaMA in fp32 (stock modules, Adam, no autocast:
/root/reference/lab/tutorial_1b/PP/1F1B/intro_PP_1F1B_MB.py:16-46,
/root/reference/lab/tutorial_1b/DP/gradient_aggr/intro_DP_GA.py:16-31). ``ops.autograd_ops`` routes
device tensors of dtype float32 here; the bf16 ops stay the opt-in fast path. Every op is
deterministic (no float atomics: slot / block partials folded in a fixed order), so an fp32 LLaMA
step gives the same bits run to run.

  linear      y = x W^T (+ b) (+ residual): FWD, DGRAD and WGRAD on the X6 planes GEMM
              (gemm_x6.hip; x, W, dY split once), dW accumulated straight into a fused grad sink;
              per (mode, shape) the tuner may pin the X6 / exact-fp32 conv engine instead (a 1x1
              conv over T "pixels"); shapes neither takes run on the exact-fp32 tabular GEMM
  rmsnorm     fork variant sums the residual branch's gradient in the backward kernel
  swiglu, embedding, causal RoPE attention, vocabulary cross-entropy
"""
from __future__ import annotations

import math
import os

import torch

from . import _lib
from . import functional as Fn
from . import functional_f32 as F32
from . import gemm_x6 as X6G
from ._lib import check, ptr, stream

vp, i32, i64, f32 = _lib.vp, _lib.i32, _lib.i64, _lib.f32
_lib.register_signatures({
    "ddl_embf_fwd": [vp, vp, vp, i32, i32, vp],
    "ddl_embf_bwd": [vp, vp, vp, i32, i32, i32, i32, vp],
    "ddl_rmsf_fwd": [vp, vp, vp, vp, i32, i32, f32, vp],
    "ddl_rmsf_blocks": [i32],
    "ddl_rmsf_bwd": [vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, vp],
    "ddl_swiglu_f32_fwd": [vp, vp, i32, i32, vp],
    "ddl_swiglu_f32_bwd": [vp, vp, vp, i32, i32, vp],
    "ddl_attnf_fwd": [vp, vp, vp, vp, vp, i32, i32, i32, i32, f32, vp],
    "ddl_attnf_bwd": [vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, f32, vp],
    "ddl_cevf": [vp, vp, i32, i32, i64, vp, i32, vp, vp, vp, i64, vp],
    "ddl_scale_f32": [vp, i64, vp, vp],
})

ATTN_HD = (16, 32, 48, 64, 96, 128)
EMB_MAX_D = 1024
RMS_MAX_D = 2048


def K():
    return _lib.kernels()


def _sink(p):
    from .autograd_ops import _grad_sink
    return _grad_sink(p)


def _ready(p):
    from .autograd_ops import _grad_ready
    _grad_ready(p)


# ------------------------------------------------------------------------------------- linear
def conv_linear_ok(C: int, Kout: int) -> bool:
    """Can the fp32 conv engine run a linear C -> Kout (FWD C % 16, DGRAD Kout % 16)?"""
    return C % 16 == 0 and Kout % 16 == 0


def x6g_ok(T: int, C: int, Kout: int) -> bool:
    """Can the planes GEMM (ops/gemm_x6.py) run a linear T x C -> Kout (every extent % 8, each
    operand's planes within the GEMM's addressing limit)?"""
    return (T % 8 == 0 and C % 8 == 0 and Kout % 8 == 0 and X6G.fits(T, C) and X6G.fits(Kout, C)
            and X6G.fits(T, Kout))


# Engine of each linear product (FWD / DGRAD / WGRAD), all native unless asked otherwise:
#   "x6g"  the X6 GEMM on pre-split planes (gemm_x6.hip): x, W and dY are split ONCE per step and
#          serve all three products (default);
#   "conv" the X6 / exact-fp32 conv engine (conv_f32.hip) as a 1x1 conv over T "pixels", where the
#          tuner measured it faster for a (mode, shape) ('lin:' entries of f32_plans.json, value
#          "conv");
#   "blas" the vendor fp32 GEMM (torch.mm -> hipBLASLt): opt-in A/B only (DDL_F32_LINEAR=blas, or
#          the older DDL_F32_BLAS=1), never chosen by default.
LINEAR = [os.environ.get("DDL_F32_LINEAR", "auto")]
_MODES = ("fwd", "dgrad", "wgrad")


def linear_engine(mode: int, T: int, C: int, Kout: int) -> str:
    if LINEAR[0] in ("x6g", "conv", "blas"):
        eng = LINEAR[0]
    elif F32.BLAS[0] == "1":
        eng = "blas"
    else:
        F32._tuned(mode, Fn.ConvGeom(1, T, 1, 1, C, Kout, 1, 1, 1, 0))  # loads the table
        eng = F32._TUNED.get(f"lin:{_MODES[mode]}:{T},{C},{Kout}", "x6g")
    if eng == "x6g" and not x6g_ok(T, C, Kout):
        eng = "conv"
    if eng == "conv" and not conv_linear_ok(C, Kout):
        eng = "tab"
    return eng


class LinearF32(torch.autograd.Function):
    """y = x W^T (+ b) (+ residual) at fp32, every product on a native kernel (see LINEAR)."""

    @staticmethod
    def forward(ctx, x, w, b, residual):
        C = x.shape[-1]
        Kout = w.shape[0]
        x2 = x.reshape(-1, C).contiguous()
        T = x2.shape[0]
        wc = w.detach().contiguous()
        eng = [linear_engine(m, T, C, Kout) for m in range(3)]
        ctx.eng = eng
        geom = Fn.ConvGeom(1, T, 1, 1, C, Kout, 1, 1, 1, 0)
        ctx.geom = geom
        # planes: x for FWD / WGRAD, W for FWD / DGRAD (split once, kept for the backward)
        px = X6G.split(x2) if "x6g" in (eng[0], eng[2]) else None
        pw = X6G.split(wc) if "x6g" in (eng[0], eng[1]) else None
        res2 = residual.reshape(T, Kout).float().contiguous() if residual is not None else None
        bias = b.detach().contiguous() if b is not None else None
        if eng[0] == "x6g":
            y = torch.empty(T, Kout, dtype=torch.float32, device=x.device)
            X6G.gemm(pw, False, px, False, y, residual=res2, bias=bias)
        elif eng[0] == "blas":
            y = torch.mm(x2, wc.t()) if res2 is None else torch.addmm(res2, x2, wc.t())
            if bias is not None:
                y.add_(bias.view(1, Kout))
        elif eng[0] == "conv":
            res = res2.view(1, T, 1, 1, Kout) if res2 is not None else None
            y = Fn.conv_fwd(x2.view(1, T, 1, 1, C), wc.view(1, Kout, 1, 1, C), geom,
                            bias=None if bias is None else bias.view(1, Kout), residual=res)
        else:
            from .tabular_ops import gemm_f32
            y = torch.empty(T, Kout, dtype=torch.float32, device=x.device)
            if res2 is not None:
                y.copy_(res2)
            gemm_f32(x2, wc, y, T, Kout, C, C, 1, 1, C, bias=bias, accumulate=res2 is not None)
        ctx.save_for_backward(x2, wc)
        ctx.px, ctx.pw = px, pw
        ctx.has_b, ctx.has_res, ctx.xshape, ctx.w = b is not None, residual is not None, x.shape, w
        return y.view(*x.shape[:-1], Kout)

    @staticmethod
    def backward(ctx, dy):
        x2, wc = ctx.saved_tensors
        T, C = x2.shape
        Kout = wc.shape[0]
        d2 = dy.reshape(T, Kout).float().contiguous()
        dx = dw = db = None
        want_dx, want_dw = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        sink = _sink(ctx.w) if want_dw else None
        eng, g = ctx.eng, ctx.geom
        ed, ew = eng[1] if want_dx else None, eng[2] if want_dw else None
        pd = X6G.split(d2) if "x6g" in (ed, ew) else None
        dy5 = d2.view(1, T, 1, 1, Kout)
        if want_dw:
            dwt = sink.view(Kout, C) if sink is not None else \
                torch.zeros(Kout, C, dtype=torch.float32, device=dy.device)
        # DGRAD and WGRAD sharing the conv engine run as one fused conv_dgrad_wgrad call
        if ed == "conv" and ew == "conv":
            dx = Fn.conv_dgrad_wgrad(dy5, wc.view(1, Kout, 1, 1, C), x2.view(1, T, 1, 1, C), g,
                                     dwt.view(1, Kout, 1, 1, C), want_dx=True)
            ed = ew = None
        if ed == "x6g":
            dx = torch.empty(T, C, dtype=torch.float32, device=dy.device)
            X6G.gemm(ctx.pw, True, pd, False, dx)
        elif ed == "blas":
            dx = torch.mm(d2, wc)
        elif ed == "conv":
            dx = Fn.conv_dgrad(dy5, wc.view(1, Kout, 1, 1, C), g)
        elif ed == "tab":
            from .tabular_ops import gemm_f32
            dx = torch.empty(T, C, dtype=torch.float32, device=dy.device)
            gemm_f32(d2, wc, dx, T, C, Kout, Kout, 1, C, 1)
        if ew == "x6g":
            X6G.gemm(ctx.px, True, pd, True, dwt, accumulate=True)
        elif ew == "blas":
            dwt.addmm_(d2.t(), x2)
        elif ew == "conv":
            Fn.conv_dgrad_wgrad(dy5, wc.view(1, Kout, 1, 1, C), x2.view(1, T, 1, 1, C), g,
                                dwt.view(1, Kout, 1, 1, C), want_dx=False)
        elif ew == "tab":
            from .tabular_ops import gemm_f32
            gemm_f32(d2, x2, dwt, Kout, C, T, 1, Kout, C, 1, accumulate=True)
        ctx.px = ctx.pw = None
        if want_dw:
            if sink is not None:
                _ready(ctx.w)
            else:
                dw = dwt
        if dx is not None:
            dx = dx.reshape(ctx.xshape)
        if ctx.has_b and ctx.needs_input_grad[2]:
            db = torch.zeros(1, Kout, dtype=torch.float32, device=dy.device)
            Fn.channel_sum(d2.view(1, T, Kout), db)
            db = db.view(Kout)
        dres = dy if ctx.has_res else None
        return dx, dw, db, dres


# ------------------------------------------------------------------------------------ rmsnorm
class RMSNormF32(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, g, eps, fork):
        D = x.shape[-1]
        x2 = x.reshape(-1, D).contiguous()
        T = x2.shape[0]
        y = torch.empty_like(x2)
        rstd = torch.empty(T, dtype=torch.float32, device=x.device)
        gd = g.detach().float().contiguous()
        check(K().ddl_rmsf_fwd(ptr(x2), ptr(gd), ptr(y), ptr(rstd), T, D, float(eps), stream()), "rmsf_fwd")
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
        want_g = ctx.needs_input_grad[1]
        sink = _sink(ctx.g) if want_g else None
        dg = sink if sink is not None else (torch.empty(D, dtype=torch.float32, device=x2.device) if want_g else None)
        dyc = torch.zeros_like(x2) if dy is None else dy.reshape(T, D).float().contiguous()
        drc = None if dres is None else dres.reshape(T, D).float().contiguous()
        part = torch.empty(int(K().ddl_rmsf_blocks(T)), D, dtype=torch.float32, device=x2.device)
        check(K().ddl_rmsf_bwd(ptr(x2), ptr(gd), ptr(rstd), ptr(dyc), ptr(drc), ptr(dx), ptr(part), ptr(dg),
                               int(sink is not None), T, D, stream()), "rmsf_bwd")
        if sink is not None:
            _ready(ctx.g)
            dg = None
        return dx.view(ctx.shape), dg, None, None


# ------------------------------------------------------------------------------------- swiglu
class SwiGLUF32(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ab):
        F2 = ab.shape[-1]
        ab2 = ab.reshape(-1, F2).contiguous()
        T = ab2.shape[0]
        h = torch.empty(T, F2 // 2, dtype=torch.float32, device=ab.device)
        check(K().ddl_swiglu_f32_fwd(ptr(ab2), ptr(h), T, F2 // 2, stream()), "swiglu_f32_fwd")
        ctx.save_for_backward(ab2)
        ctx.shape = ab.shape
        return h.view(*ab.shape[:-1], F2 // 2)

    @staticmethod
    def backward(ctx, dh):
        (ab2,) = ctx.saved_tensors
        T, F2 = ab2.shape
        dab = torch.empty_like(ab2)
        dhc = dh.reshape(T, F2 // 2).float().contiguous()
        check(K().ddl_swiglu_f32_bwd(ptr(ab2), ptr(dhc), ptr(dab), T, F2 // 2, stream()), "swiglu_f32_bwd")
        return dab.view(ctx.shape)


# ---------------------------------------------------------------------------------- embedding
class EmbeddingF32(torch.autograd.Function):
    @staticmethod
    def forward(ctx, idx, w, pad_idx):
        idx32 = idx.to(torch.int32).contiguous().reshape(-1)
        T, D = idx32.numel(), w.shape[1]
        if D > EMB_MAX_D:
            raise ValueError(f"fp32 embedding: D={D} > {EMB_MAX_D}")
        y = torch.empty(T, D, dtype=torch.float32, device=w.device)
        wd = w.detach().contiguous()
        check(K().ddl_embf_fwd(ptr(idx32), ptr(wd), ptr(y), T, D, stream()), "embf_fwd")
        ctx.save_for_backward(idx32)
        ctx.wshape, ctx.pad, ctx.w = w.shape, pad_idx, w
        return y.view(*idx.shape, D)

    @staticmethod
    def backward(ctx, dy):
        (idx32,) = ctx.saved_tensors
        V, D = ctx.wshape
        if not ctx.needs_input_grad[1]:
            return None, None, None
        sink = _sink(ctx.w)
        dw = sink if sink is not None else torch.zeros(V, D, dtype=torch.float32, device=dy.device)
        dyc = dy.reshape(-1, D).float().contiguous()
        check(K().ddl_embf_bwd(ptr(idx32), ptr(dyc), ptr(dw), idx32.numel(), D, V,
                               -1 if ctx.pad is None else int(ctx.pad), stream()), "embf_bwd")
        if sink is not None:
            _ready(ctx.w)
            dw = None
        return None, dw, None


# ---------------------------------------------------------------------------------- attention
class AttentionF32(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, H, hd):
        from .autograd_ops import rope_tables
        if hd not in ATTN_HD:
            raise ValueError(f"fp32 attention: head_dim {hd} not in {ATTN_HD}")
        B, S, _ = qkv.shape
        qc = qkv.contiguous()
        cos, sin = rope_tables(S, hd, qkv.device)
        o = torch.empty(B, S, H * hd, dtype=torch.float32, device=qkv.device)
        lse = torch.empty(B, H, S, dtype=torch.float32, device=qkv.device)
        scale = 1.0 / math.sqrt(hd)
        check(K().ddl_attnf_fwd(ptr(qc), ptr(o), ptr(lse), ptr(cos), ptr(sin), B, S, H, hd, scale, stream()),
              "attnf_fwd")
        ctx.save_for_backward(qc, o, lse)
        ctx.H, ctx.hd, ctx.scale = H, hd, scale
        return o

    @staticmethod
    def backward(ctx, do):
        from .autograd_ops import rope_tables
        qc, o, lse = ctx.saved_tensors
        B, S, _ = qc.shape
        cos, sin = rope_tables(S, ctx.hd, qc.device)
        dqkv = torch.empty_like(qc)
        delta = torch.empty_like(lse)
        doc = do.float().contiguous()
        check(K().ddl_attnf_bwd(ptr(qc), ptr(o), ptr(doc), ptr(lse), ptr(delta), ptr(dqkv), ptr(cos), ptr(sin),
                                B, S, ctx.H, ctx.hd, ctx.scale, stream()), "attnf_bwd")
        return dqkv, None, None


# ------------------------------------------------------------------------------- LM loss
class VocabCEF32(torch.autograd.Function):
    """scale x mean token CE over fp32 logits [..., V], int32 labels. The forward makes the loss
    and d(logits) at unit upstream scale in one kernel (when a gradient is needed); the backward
    rescales it in place only when the upstream gradient is not 1 (checked on the device), and a
    second backward through the same graph recomputes it first."""

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
        loss = torch.empty(1, dtype=torch.float32, device=lg.device)
        rowloss = torch.empty(R, dtype=torch.float32, device=lg.device)
        d = torch.empty_like(lg) if ctx.needs_input_grad[0] else None
        check(K().ddl_cevf(ptr(lg), ptr(lab), R, V, V, ptr(inv), int(ignore_index), ptr(rowloss), ptr(loss),
                           ptr(d), V, stream()), "cevf")
        ctx.save_for_backward(lg, lab, inv, d)
        ctx.shape, ctx.ignore, ctx.used = logits.shape, int(ignore_index), False
        return loss[0]

    @staticmethod
    def backward(ctx, g):
        lg, lab, inv, d = ctx.saved_tensors
        R, V = lg.shape
        if ctx.used:  # an earlier backward already rescaled the unit-scale gradient: recompute it
            d = torch.empty_like(lg)
            junk = torch.empty(1 + R, dtype=torch.float32, device=lg.device)
            check(K().ddl_cevf(ptr(lg), ptr(lab), R, V, V, ptr(inv), ctx.ignore, ptr(junk[1:]), ptr(junk),
                               ptr(d), V, stream()), "cevf")
        ctx.used = True
        gg = g.detach().to(torch.float32).reshape(1).contiguous()
        check(K().ddl_scale_f32(ptr(d), d.numel(), ptr(gg), stream()), "scale_f32")
        return d.view(ctx.shape), None, None, None
