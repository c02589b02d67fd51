"""Tensor-level op API over the HIP kernels (device tensors) and the PyTorch reference (CPU).

Layout contract (see csrc/include/ddl_common.h):
  * activations: bf16, NHWC, leading client-group dim  ``[G, N, H, W, C]`` (or ``[G, N, C]``);
    fp32 activations (the reference-precision mode) dispatch to ``ops.functional_f32``
  * weights: bf16 shadow views ``[G, K, R, S, C]`` whose group stride may be the flat-buffer
    stride (inner dims contiguous)
  * grads / master params / optimizer state: fp32 views of the same flat buffers
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import torch

from . import _lib
from . import autotune
from . import functional_f32 as F32
from . import reference as ref
from . import workspace as ws
from ._lib import check, ptr, stream


@dataclass(frozen=True)
class ConvGeom:
    G: int
    N: int
    H: int
    W: int
    C: int
    K: int
    R: int = 3
    S: int = 3
    stride: int = 1
    pad: int = 0

    @property
    def P(self) -> int:
        return (self.H + 2 * self.pad - self.R) // self.stride + 1

    @property
    def Q(self) -> int:
        return (self.W + 2 * self.pad - self.S) // self.stride + 1

    def flops(self) -> int:
        return 2 * self.G * self.N * self.P * self.Q * self.K * self.R * self.S * self.C


def _gs(t: torch.Tensor | None) -> int:
    return 0 if t is None else t.stride(0)


_ZERO_PAGES: dict = {}


def zero_page(device) -> torch.Tensor:
    """A small zeroed device buffer: DMA source for the implicit-GEMM padding taps."""
    key = str(device)
    z = _ZERO_PAGES.get(key)
    if z is None:
        z = torch.zeros(256, dtype=torch.float32, device=device)
        _ZERO_PAGES[key] = z
    return z


def conv_cfg(bp: int, bq: int, bk: int, ns: int, halo: bool = False) -> int:
    """Explicit conv tile choice (BP x BQ output tile, BK reduction step, NS LDS stages).
    halo: the halo-staged 3x3 / stride-1 FWD / DGRAD kernel (BK 32; tiles in ``HALO_TILES``)."""
    return (bp // 16) | ((bq // 16) << 8) | (bk << 16) | ((ns | (0x40 if halo else 0)) << 24)


CONV_TILES = [(64, 64, 32, 4), (64, 128, 32, 4), (128, 64, 32, 4), (128, 128, 32, 4),
              (128, 128, 32, 3), (64, 128, 64, 3), (128, 128, 64, 3), (128, 128, 64, 2),
              (64, 64, 64, 3), (128, 64, 64, 3), (256, 128, 32, 3), (128, 256, 32, 3),
              (256, 128, 32, 2), (128, 256, 32, 2),
              # bp = 48 selects BP = 64 with the 4 waves along Q (1x4, 64x64 per wave)
              (48, 256, 32, 4), (48, 256, 64, 3), (48, 256, 64, 2), (48, 256, 32, 3),
              # deep LDS rings for few-workgroup grids
              (64, 64, 32, 6), (64, 64, 32, 8), (64, 128, 32, 6), (64, 128, 32, 8), (128, 64, 32, 6),
              (128, 128, 32, 6)]


# halo-staged 3x3 stride-1 tiles (bp, bq, ns); bp = 48: 64 channels with the 4 waves along Q
HALO_TILES = [(48, 256, 4), (48, 128, 4), (64, 128, 4), (128, 128, 4), (128, 256, 4), (48, 256, 5),
              (48, 128, 6), (128, 128, 6)]


def halo_eligible(geom: ConvGeom, bq: int, ns: int) -> bool:
    """Mirror of conv_igemm.hip ``halo_ok``: 3x3 / stride 1 / pad 1, tiles of whole rows of one
    image or of whole images, and a halo image the taps of one channel block can DMA."""
    g = geom
    if (g.stride, g.R, g.S, g.pad) != (1, 3, 3, 1):
        return False
    hw = g.H * g.W
    if (bq % g.W or hw % bq) if hw >= bq else bq % hw:
        return False
    trh = min(bq // g.W, g.H)
    hpx = bq // (trh * g.W) * (trh + 2) * (g.W + 2)
    cap = 10 - ns if bq >= 256 else min(10 - ns, 4)
    return ((hpx + 15) // 16 + 3) // 4 <= cap


SPLITK_CAP = 1 << 24  # fp32 elements (64 MiB) of split-K partial slices per device
_SPLITK: dict = {}


def splitk_workspace(device) -> torch.Tensor | None:
    """Per-device fp32 scratch for FWD / DGRAD split-K partial sums (small grids: one client, deep
    layers). Convs on one stream use it one after another; it is allocated outside graph capture
    (the first, eager step) — a conv first seen inside a capture simply runs unsplit."""
    key = str(device)
    b = _SPLITK.get(key)
    if b is None:
        if torch.cuda.is_current_stream_capturing():
            return None
        b = torch.empty(SPLITK_CAP, dtype=torch.float32, device=device)
        _SPLITK[key] = b
    return b


def _conv_args(geom: ConvGeom, device=None, split_k: int = 0, partial: bool = False,
               **kw) -> _lib.ConvArgs:
    a = _lib.ConvArgs()
    if device is not None:
        a.zero = zero_page(device).data_ptr()
        if partial and split_k != 1:
            pw = splitk_workspace(device)
            if pw is not None:
                a.partial, a.partial_cap = pw.data_ptr(), pw.numel()
    a.split_k = split_k
    a.gscale = 1.0
    for k, v in kw.items():
        setattr(a, k, v)
    a.G, a.N, a.H, a.W, a.C, a.K = geom.G, geom.N, geom.H, geom.W, geom.C, geom.K
    a.R, a.S, a.P, a.Q, a.stride, a.pad = geom.R, geom.S, geom.P, geom.Q, geom.stride, geom.pad
    return a


def _check_inner(t: torch.Tensor, name: str) -> None:
    inner = t[0] if t.dim() > 1 else t
    if not inner.is_contiguous():
        raise ValueError(f"{name}: per-group inner dims must be contiguous")


BN_STRIPES = 32  # == BN_NSTRIPE in batchnorm.hip


def stats_buffer(G: int, C: int, device, like=None):
    """Zeroed BN statistics accumulator [G, BN_STRIPES, 2, C]: producers (conv epilogue, bn_stats)
    spread their fp32 atomics over the stripes, bn_finalize folds them. For fp32 device activations
    (``like``) a ``SlotStats`` the producing conv fills with its per-tile slots instead."""
    if like is not None and F32.is_f32(like):
        return F32.SlotStats()
    return ws.zeros((G, BN_STRIPES, 2, C), device)


def _materialize_in_bn(x, in_bn):
    """Operand-side BN (``in_bn=(scale, shift)``: the conv reads relu(x * scale + shift)) on the
    paths without the fused operand transform: apply it as a pass."""
    if in_bn is None:
        return x
    return bn_apply(x, in_bn[0], in_bn[1], act=1)


def conv_fwd(x, w, geom: ConvGeom, bias=None, relu=False, stats=None, out=None, cfg=0,
             residual=None, split_k=0, _tune=True, in_bn=None):
    """y[G,N,P,Q,K] = conv(x[G,N,H,W,C], w[G,K,R,S,C]) (+bias)(+residual)(relu);
    stats ([G,S,2,K] from ``stats_buffer``, or [G,2,K]) += per-channel sum, sumsq of y.
    split_k: 0 = automatic split-K for grids too small to fill the GPU, 1 = off, n = n slices.
    in_bn = (scale, shift): convolve relu(x * scale + shift) instead of x (fused in the fp32 kernel)."""
    if F32.is_f32(x):
        return F32.conv_fwd(x, w, geom, bias=bias, relu=relu, stats=stats, out=out, residual=residual,
                            in_bn=in_bn, split_k=split_k)
    x = _materialize_in_bn(x, in_bn)
    if not x.is_cuda:
        y = ref.conv_fwd(x, w, geom, bias, relu, stats)
        if residual is not None:
            y = (y.float() + residual.float()).to(y.dtype)
        if out is not None:
            out.copy_(y)
            return out
        return y
    _check_inner(x, "x"); _check_inner(w, "w")
    y = out if out is not None else torch.empty(geom.G, geom.N, geom.P, geom.Q, geom.K,
                                                dtype=torch.bfloat16, device=x.device)
    if residual is not None and (residual.stride(0) != y.stride(0) or not residual.is_contiguous()):
        residual = residual.contiguous()
    if _tune and cfg == 0 and split_k == 0 and autotune.ENABLED:
        def run(c, sp):
            conv_fwd(x, w, geom, bias=bias, relu=relu, out=torch.empty_like(y), cfg=c or 0,
                     stats=None if stats is None else torch.zeros_like(stats), residual=residual,
                     split_k=sp, _tune=False)
        c, split_k = autotune.pick("fwd", geom, (bias is not None, bool(relu), stats is not None,
                                                 residual is not None), run)
        cfg = c or 0
    a = _conv_args(geom, x.device, split_k, True, x=ptr(x), w=ptr(w), out=ptr(y), stats=ptr(stats), bias=ptr(bias),
                   residual=ptr(residual), x_gs=_gs(x), w_gs=_gs(w), out_gs=_gs(y),
                   bias_gs=_gs(bias), stats_gs=0 if stats is None else stats.stride(0),
                   relu=int(relu), stats_stripes=stats.shape[1] if stats is not None and stats.dim() == 4 else 1)
    check(_lib.kernels().ddl_conv_fwd(ctypes.byref(a), cfg, stream()), "conv_fwd")
    return y


def conv_dgrad(dy, w, geom: ConvGeom, residual=None, mask=None, out=None, cfg=0, bn=None, split_k=0,
               dy_bn=None, dy_bn_out=None,
               mask_bn=None, residual_sub=1, _tune=True):
    """dx[G,N,H,W,C] = conv_transpose(dy, w) (+residual) * (mask > 0).

    bn = (x, mean, rstd): also reduce, in the epilogue, the preceding BatchNorm's backward sums
    (sum dx, sum dx * (x - mean) * rstd) into a striped [G, BN_STRIPES, 2, C] buffer; returns
    (dx, part) for ``bn_backward(..., part=part)``.
    mask_bn = (scale, shift) [G, C] (with bn): the ReLU mask of ``bn_apply(x, scale, shift, relu)``
    recomputed from x in the epilogue, (x * scale + shift > 0), instead of read from its output.
    residual_sub = 2: ``residual`` is compact [G, N, ceil(H/2), ceil(W/2), C] and adds to the
    pixels (2i, 2j) only (a 1x1 / stride-2 shortcut's input gradient without its zero pixels)."""
    if mask_bn is not None:
        assert bn is not None and mask is None, "mask_bn recomputes the mask from bn's x"
    if F32.is_f32(dy):
        return F32.conv_dgrad(dy, w, geom, residual=residual, mask=mask, out=out, bn=bn, mask_bn=mask_bn,
                              residual_sub=residual_sub, split_k=split_k, dy_bn=dy_bn, dy_bn_out=dy_bn_out)
    assert dy_bn is None, "dy_bn: fp32 device activations only"
    if not dy.is_cuda:
        if mask_bn is not None:
            sc, sh = mask_bn
            xs = bn[0].float()
            bshape = (geom.G,) + (1,) * (xs.dim() - 2) + (geom.C,)
            mask = ((xs * sc.float().reshape(bshape) + sh.float().reshape(bshape)) > 0).to(dy.dtype)
        if residual is not None and residual_sub == 2:
            residual = expand_sub2(residual, geom.H, geom.W)
        dx = ref.conv_dgrad(dy, w, geom, residual, mask)
        if out is not None:
            out.copy_(dx)
            dx = out
        if bn is None:
            return dx
        x, mean, rstd = bn
        part = torch.zeros(geom.G, BN_STRIPES, 2, geom.C)
        d = dx.float().reshape(geom.G, -1, geom.C)
        xh = (x.float().reshape(geom.G, -1, geom.C) - mean[:, None]) * rstd[:, None]
        part[:, 0, 0] = d.sum(1)
        part[:, 0, 1] = (d * xh).sum(1)
        return dx, part
    _check_inner(dy, "dy"); _check_inner(w, "w")
    dx = out if out is not None else torch.empty(geom.G, geom.N, geom.H, geom.W, geom.C,
                                                 dtype=torch.bfloat16, device=dy.device)
    residual, mask = _dgrad_side_inputs(geom, dx, residual, mask, residual_sub)
    if _tune and cfg == 0 and split_k == 0 and autotune.ENABLED:
        def run(c, sp):
            conv_dgrad(dy, w, geom, residual=residual, mask=mask, out=torch.empty_like(dx), cfg=c or 0,
                       bn=bn, split_k=sp, mask_bn=mask_bn, residual_sub=residual_sub, _tune=False)
        c, split_k = autotune.pick("dgrad", geom, _dgrad_flags(residual, mask, bn, mask_bn, residual_sub), run)
        cfg = c or 0
    a, part = _dgrad_args(dy, w, geom, dx, residual, mask, bn, mask_bn, split_k, residual_sub)
    check(_lib.kernels().ddl_conv_dgrad(ctypes.byref(a), cfg, stream()), "conv_dgrad")
    return dx if bn is None else (dx, part)


def expand_sub2(r: torch.Tensor, H: int, W: int) -> torch.Tensor:
    """Compact stride-2 residual [G, N, ceil(H/2), ceil(W/2), C] -> full [G, N, H, W, C] (zeros
    off the (2i, 2j) pixels)."""
    full = torch.zeros(r.shape[0], r.shape[1], H, W, r.shape[-1], dtype=r.dtype, device=r.device)
    full[:, :, ::2, ::2] = r
    return full


def _dgrad_flags(residual, mask, bn, mask_bn, residual_sub):
    return (residual is not None, mask is not None, bn is not None, mask_bn is not None) + \
        ((True,) if residual is not None and residual_sub == 2 else ())


def _dgrad_side_inputs(geom, dx, residual, mask, residual_sub):
    if residual is not None:
        if residual_sub == 2:
            want = (geom.G, geom.N, (geom.H + 1) // 2, (geom.W + 1) // 2, geom.C)
            assert tuple(residual.shape) == want, (tuple(residual.shape), want)
            residual = residual.contiguous()
        elif residual.stride(0) != dx.stride(0):
            residual = residual.contiguous()
    if mask is not None and mask.stride(0) != dx.stride(0):
        mask = mask.contiguous()
    return residual, mask


def _dgrad_args(dy, w, geom, dx, residual, mask, bn, mask_bn, split_k, residual_sub=1):
    """ConvArgs of a DGRAD launch (+ the zeroed BN-backward partial sums when bn is fused)."""
    part = None
    kw = {}
    if bn is not None:
        x, mean, rstd = bn
        assert x.is_contiguous() and x.stride(0) == dx.stride(0) and mean.is_contiguous() and rstd.is_contiguous()
        part = ws.zeros((geom.G, BN_STRIPES, 2, geom.C), dy.device)
        kw = dict(stats=ptr(part), stats_gs=part.stride(0), stats_stripes=BN_STRIPES, bn_x=ptr(x),
                  bn_mean=ptr(mean), bn_rstd=ptr(rstd))
        if mask_bn is not None:
            sc, sh = mask_bn
            assert sc.is_contiguous() and sh.is_contiguous() and sc.numel() == geom.G * geom.C
            kw.update(mask_scale=ptr(sc), mask_shift=ptr(sh))
    if residual is not None and residual_sub == 2:
        kw.update(res_sub=2, res_gs=residual.stride(0))
    a = _conv_args(geom, dy.device, split_k, True, w=ptr(w), dy=ptr(dy), out=ptr(dx), residual=ptr(residual),
                   mask=ptr(mask), w_gs=_gs(w), dy_gs=_gs(dy), out_gs=_gs(dx), **kw)
    return a, part


def wgrad_scale(dw) -> float:
    """Scale of every WGRAD contribution into ``dw`` (ConvArgs::gscale): 1, or -lr for a view of the
    fp32 master weights handed out by ``ParamStore.grad_of`` under ``direct_update`` (the backward
    itself then applies the plain SGD step to those weights)."""
    return getattr(dw, "_ddl_wscale", 1.0)


def _wgrad_args(dy, x, geom, dw, accumulate, splits):
    gscale = wgrad_scale(dw)
    if gscale != 1.0 and not accumulate:
        raise ValueError("a scaled WGRAD must accumulate (it adds into the master weights)")
    return _conv_args(geom, dy.device, 1 if not accumulate else int(splits), x=ptr(x), dy=ptr(dy),
                      out=ptr(dw), x_gs=_gs(x), dy_gs=_gs(dy), out_gs=_gs(dw), accumulate=int(accumulate),
                      gscale=gscale)


def conv_wgrad(dy, x, geom: ConvGeom, dw, accumulate=True, cfg=0, splits=0, _tune=True, in_bn=None):
    """dw[G,K,R,S,C] (+)= sum over pixels dy (x) x  — fp32, split-K with atomics (fp32 activations:
    deterministic slices). cfg = conv_cfg(bp, bq, bk, stages) (0: tuned default); splits = split-K
    slices (0: auto). in_bn: as conv_fwd. Inside ``wgrad_overlap`` the launch goes to the side
    stream (see there)."""
    if not accumulate and wgrad_scale(dw) != 1.0:
        raise ValueError("a scaled WGRAD must accumulate (it adds into the master weights)")
    if F32.is_f32(dy):
        side = _WGRAD_SIDE
        if side is None:
            return F32.conv_wgrad(dy, x, geom, dw, accumulate, wgrad_scale(dw), in_bn=in_bn, split_k=splits)
        # side stream: after everything queued so far (the DGRAD that reads the weights this
        # direct-SGD WGRAD steps), concurrent with the rest of the backward; joined on exit of
        # wgrad_overlap. Its split-K workspace is the side stream's own (functional_f32.workspace).
        side.wait_stream(torch.cuda.current_stream())
        # keep the inputs alive until wgrad_overlap joins the side stream back (not record_stream:
        # inside a graph capture the allocator can never retire a record_stream'd block, so every
        # captured step would grow the graph's private pool — 226 GiB reserved for one 8-client round)
        _side_keep(side, (dy, x) + (tuple(in_bn) if in_bn is not None else ()))
        with torch.cuda.stream(side):
            return F32.conv_wgrad(dy, x, geom, dw, accumulate, wgrad_scale(dw), in_bn=in_bn, split_k=splits,
                                  ws_role="side")
    x = _materialize_in_bn(x, in_bn)
    if not dy.is_cuda:
        ref.conv_wgrad(dy, x, geom, dw, accumulate, wgrad_scale(dw))
        return dw
    _check_inner(dy, "dy"); _check_inner(x, "x"); _check_inner(dw, "dw")
    if _tune and cfg == 0 and splits == 0 and autotune.ENABLED:
        def run(c, sp):
            global _WGRAD_SIDE
            side, _WGRAD_SIDE = _WGRAD_SIDE, None  # timed on the current stream
            try:
                conv_wgrad(dy, x, geom, torch.zeros_like(dw), accumulate, cfg=c or 0, splits=sp, _tune=False)
            finally:
                _WGRAD_SIDE = side
        c, splits = autotune.pick("wgrad", geom, (bool(accumulate),), run, accumulate=bool(accumulate))
        cfg = c or 0
    a = _wgrad_args(dy, x, geom, dw, accumulate, splits)
    side = _WGRAD_SIDE
    if side is None:
        check(_lib.kernels().ddl_conv_wgrad(ctypes.byref(a), cfg, stream()), "conv_wgrad")
        return dw
    side.wait_stream(torch.cuda.current_stream())
    _side_keep(side, (dy, x))  # as the fp32 branch: no record_stream (graph-pool growth)
    with torch.cuda.stream(side):
        check(_lib.kernels().ddl_conv_wgrad(ctypes.byref(a), cfg, stream()), "conv_wgrad")
    return dw


# ------------------------------------------------------------------- wgrad / dgrad overlap
_WGRAD_SIDE: "torch.cuda.Stream | None" = None
_SIDE_STREAMS: dict = {}
# side-stream WGRAD inputs per side stream, released when wgrad_overlap joins THAT stream back
_SIDE_KEEP: dict = {}


def _side_keep(side, tensors) -> None:
    _SIDE_KEEP.setdefault(side.cuda_stream, []).extend(tensors)


# Paired DGRAD + WGRAD of one conv in one launch (conv_igemm.hip ``ddl_conv_pair``). The pair
# tuner (autotune.pick_pair) times it against the two tuned single launches per shape; DDL_CONV_PAIR=0
# keeps the single launches everywhere.
PAIR_ENABLED = __import__("os").environ.get("DDL_CONV_PAIR", "1") != "0"
# the paired kernels' tile menu (mirrors the TileOp list of conv_igemm.hip)
PAIR_DGRAD = [(48, 256, 32, 4, True), (48, 128, 32, 4, True), (128, 128, 64, 2, False),
              (64, 128, 64, 3, False), (128, 64, 64, 3, False), (48, 256, 64, 2, False)]
PAIR_WGRAD = [(64, 64, 64, 3), (128, 64, 64, 3), (128, 128, 32, 3), (128, 128, 64, 2), (64, 128, 32, 4)]
MODE_FWD, MODE_DGRAD, MODE_WGRAD = 0, 1, 2


def conv_pair(dy, w, x, geom: ConvGeom, dw, dcfg: int, dsplit: int, wcfg: int, wsplit: int,
              residual=None, mask=None, bn=None, mask_bn=None, out=None, residual_sub=1, dgeom=None):
    """Explicit paired launch: DGRAD (tile ``dcfg``, split ``dsplit``, fused epilogue as conv_dgrad;
    geometry ``dgeom`` or ``geom``) and WGRAD (``wcfg``, ``wsplit``, accumulating into dw) in one
    grid. -> (dx, part | None). Raises KernelError when the tiles have no paired instantiation."""
    dg = dgeom or geom
    dx = out if out is not None else torch.empty(dg.G, dg.N, dg.H, dg.W, dg.C,
                                                 dtype=torch.bfloat16, device=dy.device)
    residual, mask = _dgrad_side_inputs(dg, dx, residual, mask, residual_sub)
    ad, part = _dgrad_args(dy, w, dg, dx, residual, mask, bn, mask_bn, dsplit, residual_sub)
    aw = _wgrad_args(dy, x, geom, dw, True, wsplit)
    rc = _lib.kernels().ddl_conv_pair(ctypes.byref(ad), MODE_DGRAD, dcfg, ctypes.byref(aw), MODE_WGRAD,
                                      wcfg, stream())
    if rc == -1:
        raise _lib.KernelError("no paired kernel for these tiles")
    check(rc, "conv_pair")
    return dx, part


def conv_dgrad_wgrad(dy, w, x, geom: ConvGeom, dw, residual=None, mask=None, bn=None, mask_bn=None,
                     want_dx: bool = True, residual_sub: int = 1, dgeom: ConvGeom | None = None, in_bn=None,
                     dy_bn=None):
    """``conv_wgrad(dy, x, geom, dw)`` and (if want_dx) ``conv_dgrad(dy, w, dgeom or geom, residual,
    mask, bn=bn, mask_bn=mask_bn, residual_sub=...)`` — both read dy and are independent, so on
    the GPU they may run as ONE paired launch (whichever of paired / back-to-back the tuner
    measured faster for this shape). ``dgeom``: the DGRAD's own geometry (a stride-2 1x1
    shortcut's input gradient on the compact grid). Returns what conv_dgrad returns (None
    without want_dx). in_bn: the WGRAD's operand-side BN of x (as conv_fwd). dy_bn = (x_bn, coef)
    (fp32): dY is the following BN's backward A * dy + B * x_bn + C, applied inside the DGRAD as it
    stages dY (which also writes it out for the WGRAD) instead of by a separate apply pass."""
    dg = dgeom or geom
    dkw = dict(residual=residual, mask=mask, bn=bn, mask_bn=mask_bn, residual_sub=residual_sub)
    if dy_bn is not None:
        assert F32.is_f32(dy) and dgeom is None
        if want_dx:
            dc = torch.empty_like(dy)
            dx = conv_dgrad(dy, w, dg, dy_bn=dy_bn, dy_bn_out=dc, **dkw)
        else:
            dc, dx = F32.coef_apply(dy, dy_bn[0], dy_bn[1]), None
        conv_wgrad(dc, x, geom, dw, in_bn=in_bn)
        return dx
    if F32.is_f32(dy) or in_bn is not None:
        # DGRAD first: in fp32 ``w`` IS the master weight that a direct-SGD WGRAD steps in place
        dx = conv_dgrad(dy, w, dg, **dkw) if want_dx else None
        conv_wgrad(dy, x, geom, dw, in_bn=in_bn)
        return dx
    if not want_dx or not dy.is_cuda or not PAIR_ENABLED or _WGRAD_SIDE is not None \
            or not autotune.ENABLED:
        conv_wgrad(dy, x, geom, dw)
        if not want_dx:
            return None
        return conv_dgrad(dy, w, dg, **dkw)
    _check_inner(dy, "dy"); _check_inner(w, "w"); _check_inner(x, "x"); _check_inner(dw, "dw")
    dx = torch.empty(dg.G, dg.N, dg.H, dg.W, dg.C, dtype=torch.bfloat16, device=dy.device)
    residual, mask = _dgrad_side_inputs(dg, dx, residual, mask, residual_sub)
    dkw.update(residual=residual, mask=mask)
    dflags = _dgrad_flags(residual, mask, bn, mask_bn, residual_sub)
    lib = _lib.kernels()

    def run_d(c, sp):
        return conv_dgrad(dy, w, dg, out=torch.empty_like(dx), cfg=c or 0, split_k=sp, _tune=False, **dkw)

    def run_w(c, sp):
        conv_wgrad(dy, x, geom, torch.zeros_like(dw), True, cfg=c or 0, splits=sp, _tune=False)

    dpick = autotune.pick("dgrad", dg, dflags, run_d)
    wpick = autotune.pick("wgrad", geom, (True,), run_w)

    def supported(dc, dsp, wc, wsp):
        ad, _ = _dgrad_args(dy, w, dg, dx, residual, mask, bn, mask_bn, dsp, residual_sub)
        aw = _wgrad_args(dy, x, geom, dw, True, wsp)
        return bool(lib.ddl_conv_pair_supported(ctypes.byref(ad), MODE_DGRAD, dc or 0,
                                                ctypes.byref(aw), MODE_WGRAD, wc or 0))

    def launch_pair(cand, dx_out, dw_out):
        dc, dsp, wc, wsp = cand
        return conv_pair(dy, w, x, geom, dw_out, dc or 0, dsp, wc or 0, wsp, out=dx_out, dgeom=dgeom,
                         **dkw)[1]

    def run_seq():
        run_w(*wpick)
        run_d(*dpick)

    tag = ("pair", dflags) + ((dg.H, dg.W, dg.R, dg.stride) if dgeom is not None else ())
    choice = autotune.pick_pair(tag, geom, dpick, wpick, supported,
                                lambda cand: launch_pair(cand, torch.empty_like(dx), torch.zeros_like(dw)),
                                run_seq,
                                [(conv_cfg(bp, bq, bk, ns, h), 0) for bp, bq, bk, ns, h in PAIR_DGRAD],
                                [(conv_cfg(*t), 0) for t in PAIR_WGRAD])
    if choice is None:  # back-to-back single launches
        conv_wgrad(dy, x, geom, dw, cfg=wpick[0] or 0, splits=wpick[1], _tune=False)
        return conv_dgrad(dy, w, dg, out=dx, cfg=dpick[0] or 0, split_k=dpick[1], _tune=False, **dkw)
    part = launch_pair(choice, dx, dw)
    return dx if bn is None else (dx, part)


# Paired FWD + FWD (a downsample block's last 3x3 conv, A, and its 1x1 projection shortcut, B)
PAIR_FWD_A = [(64, 64, 64, 3), (64, 128, 64, 3), (128, 128, 32, 3), (128, 64, 64, 3)]
PAIR_FWD_B = [(64, 128, 32, 4), (64, 64, 64, 3), (64, 128, 64, 3)]
PAIR_FWD_ENABLED = __import__("os").environ.get("DDL_CONV_PAIR_FWD", "1") != "0"


def _fwd_pair_args(x, w, geom, y, stats, split_k, partial):
    return _conv_args(geom, x.device, split_k, partial, x=ptr(x), w=ptr(w), out=ptr(y), stats=ptr(stats),
                      x_gs=_gs(x), w_gs=_gs(w), out_gs=_gs(y),
                      stats_gs=0 if stats is None else stats.stride(0),
                      stats_stripes=stats.shape[1] if stats is not None and stats.dim() == 4 else 1)


def conv_fwd_pair(xa, wa, ga: ConvGeom, stats_a, acfg: int, asplit: int, xb, wb, gb: ConvGeom, stats_b,
                  bcfg: int, out_a=None, out_b=None, check_only: bool = False):
    """Explicit paired launch of two independent FWD convs (tiles ``acfg`` / ``bcfg``, 0 = the
    heuristic; op A may split-K with ``asplit``, op B never does: the split workspace is one per
    device) -> (ya, yb). Raises KernelError when the tiles have no paired instantiation;
    ``check_only`` -> whether they have one (nothing launched)."""
    dev = xa.device
    ya = out_a if out_a is not None else torch.empty(ga.G, ga.N, ga.P, ga.Q, ga.K, dtype=torch.bfloat16, device=dev)
    yb = out_b if out_b is not None else torch.empty(gb.G, gb.N, gb.P, gb.Q, gb.K, dtype=torch.bfloat16, device=dev)
    a = _fwd_pair_args(xa, wa, ga, ya, stats_a, asplit, True)
    b = _fwd_pair_args(xb, wb, gb, yb, stats_b, 1, False)
    lib = _lib.kernels()
    if check_only:
        return bool(lib.ddl_conv_pair_supported(ctypes.byref(a), MODE_FWD, acfg, ctypes.byref(b), MODE_FWD, bcfg))
    rc = lib.ddl_conv_pair(ctypes.byref(a), MODE_FWD, acfg, ctypes.byref(b), MODE_FWD, bcfg, stream())
    if rc == -1:
        raise _lib.KernelError("no paired kernel for these tiles")
    check(rc, "conv_pair")
    return ya, yb


def conv_fwd2(xa, wa, ga: ConvGeom, stats_a, xb, wb, gb: ConvGeom, stats_b):
    """Two independent convolutions, each ``conv_fwd(x, w, geom, stats=stats)`` -> (ya, yb): a
    downsample block's last conv (A) and its projection shortcut on the block input (B). On the
    GPU they may run as ONE paired launch (whichever of paired / back-to-back the pair tuner
    measured faster for these shapes)."""
    if not xa.is_cuda or F32.is_f32(xa) or not PAIR_ENABLED or not PAIR_FWD_ENABLED or not autotune.ENABLED:
        return conv_fwd(xa, wa, ga, stats=stats_a), conv_fwd(xb, wb, gb, stats=stats_b)
    _check_inner(xa, "xa"); _check_inner(wa, "wa"); _check_inner(xb, "xb"); _check_inner(wb, "wb")
    dev = xa.device
    ya = torch.empty(ga.G, ga.N, ga.P, ga.Q, ga.K, dtype=torch.bfloat16, device=dev)
    yb = torch.empty(gb.G, gb.N, gb.P, gb.Q, gb.K, dtype=torch.bfloat16, device=dev)
    fa, fb = (False, False, stats_a is not None, False), (False, False, stats_b is not None, False)

    def scratch(st):
        return None if st is None else torch.zeros_like(st)

    def run_a(c, sp):
        conv_fwd(xa, wa, ga, out=torch.empty_like(ya), cfg=c or 0, stats=scratch(stats_a), split_k=sp, _tune=False)

    def run_b(c, sp):
        conv_fwd(xb, wb, gb, out=torch.empty_like(yb), cfg=c or 0, stats=scratch(stats_b), split_k=sp, _tune=False)

    apick = autotune.pick("fwd", ga, fa, run_a)
    bpick = autotune.pick("fwd", gb, fb, run_b)

    def pair(cand, **kw):
        ac, asp, bc, _ = cand
        return conv_fwd_pair(xa, wa, ga, kw.pop("sa", stats_a), ac or 0, asp, xb, wb, gb,
                             kw.pop("sb", stats_b), bc or 0, **kw)

    def run_seq():
        run_a(*apick)
        run_b(*bpick)

    tag = ("fwd2", fa, fb, gb.N, gb.H, gb.W, gb.C, gb.K, gb.R, gb.S, gb.stride, gb.pad)
    choice = autotune.pick_pair(tag, ga, apick, bpick,
                                lambda *cand: pair(cand, out_a=ya, out_b=yb, check_only=True),
                                lambda cand: pair(cand, sa=scratch(stats_a), sb=scratch(stats_b)),
                                run_seq,
                                [(conv_cfg(*t), 0) for t in PAIR_FWD_A],
                                [(conv_cfg(*t), 0) for t in PAIR_FWD_B])
    if choice is None:  # back-to-back single launches
        conv_fwd(xa, wa, ga, out=ya, cfg=apick[0] or 0, stats=stats_a, split_k=apick[1], _tune=False)
        conv_fwd(xb, wb, gb, out=yb, cfg=bpick[0] or 0, stats=stats_b, split_k=bpick[1], _tune=False)
        return ya, yb
    return pair(choice, out_a=ya, out_b=yb)


class wgrad_overlap:
    """Backward-pass stream split: inside this context every ``conv_wgrad`` runs on a side stream
    (after an event on the main stream), so a layer's weight gradient can overlap the main
    stream's dgrad -> BN-backward chain of the layers below it (the two are independent: wgrad
    only accumulates into the fp32 grad buffer). Leaving the context joins the side stream back;
    captured in a HIP graph this is a fork/join per layer. ``Net.overlap_wgrad`` turns it on for
    fp32 nets (measured faster) and off for bf16 ones (the cross-queue synchronisation cost more
    than the overlap won on the graph-replayed bf16 ResNet-18 step).
    ``run_joined(fn)`` runs ``fn`` (e.g. a DP all-reduce hook) ordered after both streams."""

    def __init__(self, device, enabled: bool = True):
        self.enabled = enabled and torch.device(device).type == "cuda"
        self.device = torch.device(device)

    def __enter__(self):
        global _WGRAD_SIDE
        self.prev = _WGRAD_SIDE
        if self.enabled:
            key = str(self.device)
            if key not in _SIDE_STREAMS:
                _SIDE_STREAMS[key] = torch.cuda.Stream(self.device)
            _WGRAD_SIDE = _SIDE_STREAMS[key]
        return self

    def __exit__(self, *exc):
        global _WGRAD_SIDE
        if _WGRAD_SIDE is not None and _WGRAD_SIDE is not self.prev:
            torch.cuda.current_stream().wait_stream(_WGRAD_SIDE)
            # joined: this side stream's inputs may be reused in stream order (other devices'
            # side streams, not joined here, keep theirs)
            _SIDE_KEEP.pop(_WGRAD_SIDE.cuda_stream, None)
        _WGRAD_SIDE = self.prev
        return False

    @staticmethod
    def run_joined(fn):
        side = _WGRAD_SIDE
        if side is None:
            return fn()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            return fn()


# ------------------------------------------------------------------------------------- BN
def bn_finalize(stats, gamma, beta, running_mean, running_var, count, eps=1e-5, momentum=0.1,
                training=True):
    """-> (scale, shift, mean, rstd), each [G, C] fp32 contiguous."""
    if isinstance(stats, F32.SlotStats):
        G = stats.t.shape[0] if stats.t is not None else running_mean.shape[0]
        C = stats.t.shape[-1] if stats.t is not None else running_mean.shape[-1]
        return F32.bn_finalize_many([(stats, gamma, beta, running_mean, running_var, count, G, C)], eps, momentum,
                                    training)[0]
    if not stats.is_cuda:
        return ref.bn_finalize(stats, gamma, beta, running_mean, running_var, count, eps, momentum,
                               training)
    G, C = stats.shape[0], stats.shape[-1]
    outs = torch.empty(4, G, C, dtype=torch.float32, device=stats.device)
    a = _lib.BNArgs()
    a.stats, a.gamma, a.beta = ptr(stats), ptr(gamma), ptr(beta)
    a.running_mean, a.running_var = ptr(running_mean), ptr(running_var)
    a.scale, a.shift, a.mean, a.rstd = (ptr(outs[i]) for i in range(4))
    a.gs_param = _gs(gamma) if gamma is not None else _gs(beta)
    a.gs_buf = _gs(running_mean)
    a.G, a.C, a.count = G, C, int(count)
    a.eps, a.momentum, a.training = float(eps), float(momentum), int(training)
    a.stripes = stats.shape[1] if stats.dim() == 4 else 1
    assert stats.is_contiguous()
    check(_lib.kernels().ddl_bn_finalize(ctypes.byref(a), stream()), "bn_finalize")
    return outs[0], outs[1], outs[2], outs[3]


def _bn_fin_args(stats, gamma, beta, running_mean, running_var, count, eps, momentum, outs):
    G, C = stats.shape[0], stats.shape[-1]
    a = _lib.BNArgs()
    a.stats, a.gamma, a.beta = ptr(stats), ptr(gamma), ptr(beta)
    a.running_mean, a.running_var = ptr(running_mean), ptr(running_var)
    a.scale, a.shift, a.mean, a.rstd = (ptr(outs[i]) for i in range(4))
    a.gs_param = _gs(gamma) if gamma is not None else _gs(beta)
    a.gs_buf = _gs(running_mean)
    a.G, a.C, a.count = G, C, int(count)
    a.eps, a.momentum, a.training = float(eps), float(momentum), 1
    a.stripes = stats.shape[1] if stats.dim() == 4 else 1
    assert stats.is_contiguous()
    return a


def bn_finalize2(bn_a, bn_b, eps=1e-5, momentum=0.1):
    """Training-mode bn_finalize of two independent BatchNorms in one launch (a residual block's
    output BN and its projected shortcut's BN). bn_* = (stats, gamma, beta, running_mean,
    running_var, count) -> ((scale, shift, mean, rstd), (scale, shift, mean, rstd))."""
    if isinstance(bn_a[0], F32.SlotStats):
        items = [(bn[0], *bn[1:], bn[0].t.shape[0], bn[0].t.shape[-1]) for bn in (bn_a, bn_b)]
        return tuple(F32.bn_finalize_many(items, eps, momentum))
    if not bn_a[0].is_cuda:
        return (bn_finalize(*bn_a, eps, momentum), bn_finalize(*bn_b, eps, momentum))
    outs = []
    for bn in (bn_a, bn_b):
        G, C = bn[0].shape[0], bn[0].shape[-1]
        outs.append(torch.empty(4, G, C, dtype=torch.float32, device=bn[0].device))
    a = _bn_fin_args(*bn_a, eps, momentum, outs[0])
    b = _bn_fin_args(*bn_b, eps, momentum, outs[1])
    check(_lib.kernels().ddl_bn_finalize2(ctypes.byref(a), ctypes.byref(b), stream()), "bn_finalize2")
    return tuple(outs[0]), tuple(outs[1])


def bn_bwd_reduce_part(dy, ymask, x, mean, rstd):
    """Striped BN backward reduce sums [G, BN_STRIPES, 2, C] (sum dy_m, sum dy_m * xhat) for
    ``bn_backward(..., part=)`` / ``bn_backward2``; dy_m = dy * (ymask > 0) (ymask nullable)."""
    G, C = x.shape[0], x.shape[-1]
    if F32.is_f32(dy):
        return F32.bn_bwd_reduce_part(dy, ymask, x, mean, rstd)
    if not dy.is_cuda:
        sums = ref.bn_bwd_reduce(dy, ymask, x, mean, rstd)
        part = torch.zeros(G, BN_STRIPES, 2, C)
        part[:, 0] = sums
        return part
    part = ws.zeros((G, BN_STRIPES, 2, C), x.device)
    check(_lib.kernels().ddl_bn_bwd_reduce_part(ptr(dy), ptr(ymask), ptr(x), ptr(mean), ptr(rstd),
                                                ptr(part), x[0].numel() // C, C, G, stream()),
          "bn_bwd_reduce_part")
    return part


def bn_backward2(dy, bn_a, bn_b):
    """Two BatchNorm backwards sharing the already-masked input gradient dy (a block's output BN and
    its shortcut's BN): one fold launch for both and one apply pass that reads dy once.
    bn_* = (x, mean, rstd, gamma, dgamma, dbeta, part) -> (dx_a, dx_b)."""
    if F32.is_f32(dy):
        return F32.bn_backward2(dy, bn_a, bn_b)
    if not dy.is_cuda:
        return tuple(bn_backward(dy, None, bn[0], bn[1], bn[2], bn[3], bn[4], bn[5], part=bn[6])
                     for bn in (bn_a, bn_b))
    xa = bn_a[0]
    G, C = xa.shape[0], xa.shape[-1]
    assert bn_b[0].shape == xa.shape and dy.is_contiguous()
    args, outs = [], []
    for x, mean, rstd, gamma, dgamma, dbeta, part in (bn_a, bn_b):
        t = _lib.BNBwdArgs()
        dx = torch.empty_like(x)
        coef = ws.scratch((G, 3, C), x.device)
        gs = _gs(gamma) if gamma is not None else 0
        if dgamma is not None or dbeta is not None:
            gs = _gs(dgamma) if dgamma is not None else _gs(dbeta)
        t.x, t.mean, t.rstd, t.gamma = ptr(x), ptr(mean), ptr(rstd), ptr(gamma)
        t.dgamma, t.dbeta, t.part, t.coef, t.dx, t.gs_param = ptr(dgamma), ptr(dbeta), ptr(part), \
            ptr(coef), ptr(dx), gs
        t._keep = coef  # outside a step's arena the scratch must outlive the launch
        args.append(t)
        outs.append(dx)
    check(_lib.kernels().ddl_bn_backward2(ptr(dy), ctypes.byref(args[0]), ctypes.byref(args[1]),
                                          xa[0].numel() // C, C, G, stream()), "bn_backward2")
    return outs[0], outs[1]


def bn_apply(x, scale, shift, r=None, rscale=None, rshift=None, act=0, out=None):
    if F32.is_f32(x):
        return F32.bn_apply(x, scale, shift, r, rscale, rshift, act, out)
    if not x.is_cuda:
        y = ref.bn_apply(x, scale, shift, r, rscale, rshift, act)
        if out is not None:
            out.copy_(y)
            return out
        return y
    assert x.is_contiguous() and (r is None or r.is_contiguous())
    y = out if out is not None else torch.empty_like(x)
    G, C = x.shape[0], x.shape[-1]
    check(_lib.kernels().ddl_bn_apply(ptr(x), ptr(scale), ptr(shift), ptr(r), ptr(rscale),
                                      ptr(rshift), ptr(y), x[0].numel(), C, G, act, stream()),
          "bn_apply")
    return y


def bn_stats(x, stats=None):
    """stats [G, BN_STRIPES, 2, C] fp32 (+)= per-channel (sum, sum of squares) of x [G, ..., C]."""
    G, C = x.shape[0], x.shape[-1]
    if F32.is_f32(x):
        assert stats is None, "fp32 statistics are returned as a new SlotStats"
        return F32.bn_stats(x)
    if stats is None:
        stats = stats_buffer(G, C, x.device)
    if not x.is_cuda:
        ref.bn_stats(x, stats)
        return stats
    assert x.is_contiguous() and x.dtype == torch.bfloat16 and stats.shape[1] == BN_STRIPES
    check(_lib.kernels().ddl_bn_stats(ptr(x), ptr(stats), x[0].numel() // C, C, G, stream()),
          "bn_stats")
    return stats


def bn_bwd_reduce(dy, ymask, x, mean, rstd, dgamma=None, dbeta=None):
    """-> sums [G, 2, C] = (sum dy_m, sum dy_m*xhat); also accumulates into dgamma/dbeta views."""
    assert not F32.is_f32(dy), "fp32 activations: use bn_backward / bn_bwd_reduce_part"
    if not dy.is_cuda:
        return ref.bn_bwd_reduce(dy, ymask, x, mean, rstd, dgamma, dbeta)
    G, C = x.shape[0], x.shape[-1]
    part = ws.zeros((G, BN_STRIPES, 2, C), x.device)
    sums = ws.scratch((G, 2, C), x.device)
    gs = _gs(dgamma) if dgamma is not None else _gs(dbeta)
    check(_lib.kernels().ddl_bn_bwd_reduce(ptr(dy), ptr(ymask), ptr(x), ptr(mean), ptr(rstd),
                                           ptr(part), ptr(sums), ptr(dgamma), ptr(dbeta), gs,
                                           x[0].numel() // C, C, G, stream()), "bn_bwd_reduce")
    return sums


def bn_backward(dy, ymask, x, mean, rstd, gamma, dgamma=None, dbeta=None, emit_dym=False,
                part=None):
    """Whole BN backward (= bn_bwd_reduce + bn_bwd_apply) in three launches; accumulates
    d(gamma), d(beta) into the given [G, C] views. -> dx (, dy_m if emit_dym).
    ``part``: the striped reduce sums already produced by dy's producer (``conv_dgrad(bn=...)``,
    which also applied the mask) — the reduce pass is skipped (two launches)."""
    if F32.is_f32(dy):
        return F32.bn_backward(dy, ymask, x, mean, rstd, gamma, dgamma, dbeta, emit_dym, part)
    if not dy.is_cuda:
        if part is not None:
            sums = part.sum(1)
            if dbeta is not None:
                dbeta += sums[:, 0]
            if dgamma is not None:
                dgamma += sums[:, 1]
        else:
            sums = ref.bn_bwd_reduce(dy, ymask, x, mean, rstd, dgamma, dbeta)
        return ref.bn_bwd_apply(dy, ymask, x, mean, rstd, gamma, sums, emit_dym)
    G, C = x.shape[0], x.shape[-1]
    do_reduce = part is None
    if part is None:
        part = ws.zeros((G, BN_STRIPES, 2, C), x.device)
    coef = ws.scratch((G, 3, C), x.device)
    dx = torch.empty_like(x)
    dym = torch.empty_like(x) if emit_dym else None
    gs = _gs(gamma) if gamma is not None else 0
    if dgamma is not None or dbeta is not None:
        gd = _gs(dgamma) if dgamma is not None else _gs(dbeta)
        assert gamma is None or gd == gs, "gamma and its gradient must share the group stride"
        gs = gd
    check(_lib.kernels().ddl_bn_backward(ptr(dy), ptr(ymask), ptr(x), ptr(mean), ptr(rstd),
                                         ptr(gamma), gs, ptr(part), ptr(coef), ptr(dgamma),
                                         ptr(dbeta), ptr(dx), ptr(dym), x[0].numel() // C, C, G,
                                         int(do_reduce), stream()), "bn_backward")
    return (dx, dym) if emit_dym else dx


def bn_bwd_apply(dy, ymask, x, mean, rstd, gamma, sums, emit_dym=False):
    assert not F32.is_f32(dy), "fp32 activations: use bn_backward"
    if not dy.is_cuda:
        return ref.bn_bwd_apply(dy, ymask, x, mean, rstd, gamma, sums, emit_dym)
    G, C = x.shape[0], x.shape[-1]
    dx = torch.empty_like(x)
    dym = torch.empty_like(x) if emit_dym else None
    coef = ws.scratch((G, 3, C), x.device)
    check(_lib.kernels().ddl_bn_bwd_apply(ptr(dy), ptr(ymask), ptr(x), ptr(mean), ptr(rstd),
                                          ptr(gamma), _gs(gamma), ptr(sums), ptr(coef), ptr(dx),
                                          ptr(dym), x[0].numel() // C, C, G, stream()),
          "bn_bwd_apply")
    return (dx, dym) if emit_dym else dx


# ----------------------------------------------------------------------------- elementwise
def _k(name: str, t: torch.Tensor):
    """The launcher for t's activation dtype: ``name`` (bf16) or its ``_f32`` twin."""
    lib = _lib.kernels()
    if t.dtype == torch.float32:
        return getattr(lib, name + "_f32")
    assert t.dtype == torch.bfloat16, f"{name}: unsupported activation dtype {t.dtype}"
    return getattr(lib, name)


def maxpool2_fwd(x):
    if not x.is_cuda:
        return ref.maxpool2_fwd(x)
    G, N, H, W, C = x.shape
    y = torch.empty(G, N, H // 2, W // 2, C, dtype=x.dtype, device=x.device)
    check(_k("ddl_maxpool2_fwd", x)(ptr(x), ptr(y), G * N, H, W, C, stream()), "maxpool2_fwd")
    return y


def maxpool2_bwd(x, dy):
    if not x.is_cuda:
        return ref.maxpool2_bwd(x, dy)
    G, N, H, W, C = x.shape
    dx = torch.empty_like(x)
    check(_k("ddl_maxpool2_bwd", x)(ptr(x), ptr(dy), ptr(dx), G * N, H, W, C, stream()),
          "maxpool2_bwd")
    return dx


def avgpool_fwd(x):
    if not x.is_cuda:
        return ref.avgpool_fwd(x)
    G, N, H, W, C = x.shape
    y = torch.empty(G, N, C, dtype=x.dtype, device=x.device)
    check(_k("ddl_avgpool_fwd", x)(ptr(x), ptr(y), G * N, H * W, C, stream()), "avgpool_fwd")
    return y


def avgpool_bwd(dy, H, W):
    if not dy.is_cuda:
        return ref.avgpool_bwd(dy, H, W)
    G, N, C = dy.shape
    dx = torch.empty(G, N, H, W, C, dtype=dy.dtype, device=dy.device)
    check(_k("ddl_avgpool_bwd", dy)(ptr(dy), ptr(dx), G * N, H * W, C, stream()), "avgpool_bwd")
    return dx


def avgpool_bwd_bn(dy, x, bn):
    """Global-average-pool backward for a pooled input x = relu(BN(c) [+ r]) fused with that BN's
    backward reduce: -> (dx = dy/HW * (x > 0), part [G, BN_STRIPES, 2, C] with (sum dx,
    sum dx * (c - mean) * rstd)) for ``bn_backward(..., part=part)``. bn = (c, mean, rstd)."""
    if F32.is_f32(x):
        return F32.avgpool_bwd_bn(dy, x, bn)
    c, mean, rstd = bn
    G, N, H, W, C = x.shape
    if not dy.is_cuda:
        d = dy.float().reshape(G, N, 1, 1, C) / (H * W) * (x.float() > 0)
        dx = d.to(dy.dtype).contiguous()
        xh = (c.float() - mean.reshape(G, 1, 1, 1, C)) * rstd.reshape(G, 1, 1, 1, C)
        part = torch.zeros(G, BN_STRIPES, 2, C)
        df = dx.float()
        part[:, 0, 0] = df.reshape(G, -1, C).sum(1)
        part[:, 0, 1] = (df * xh).reshape(G, -1, C).sum(1)
        return dx, part
    assert x.is_contiguous() and c.is_contiguous() and dy.is_contiguous()
    dx = torch.empty_like(x)
    part = ws.zeros((G, BN_STRIPES, 2, C), x.device)
    check(_lib.kernels().ddl_avgpool_bwd_bn(ptr(dy), ptr(x), ptr(c), ptr(mean), ptr(rstd), ptr(dx),
                                            ptr(part), G, N, H * W, C, stream()), "avgpool_bwd_bn")
    return dx, part


def dropout(x, p, seed, offset, offset_dev=None):
    """Philox dropout; the counter base is ``offset`` (+ the int64 device scalar ``offset_dev``)."""
    if p <= 0:
        return x
    if not x.is_cuda:
        extra = int(offset_dev.item()) if offset_dev is not None else 0
        return ref.dropout(x, p, seed, offset + extra)
    y = torch.empty_like(x)
    check(_k("ddl_dropout", x)(ptr(x), ptr(y), x.numel(), float(p), int(seed), int(offset),
                                     ptr(offset_dev), stream()), "dropout")
    return y


def u64_add(t, inc: int):
    """t (int64 device scalar) += inc, stream-ordered (graph-capturable)."""
    if not t.is_cuda:
        t += inc
        return t
    check(_lib.kernels().ddl_u64_add(ptr(t), int(inc), stream()), "u64_add")
    return t


ACT = {"none": 0, "relu": 1, "leaky_relu": 2, "tanh": 3, "sigmoid": 4}


def act_fwd(x, act: int, slope=0.01):
    if not x.is_cuda:
        return ref.act_fwd(x, act, slope)
    y = torch.empty_like(x)
    check(_k("ddl_act_fwd", x)(ptr(x), ptr(y), x.numel(), act, float(slope), stream()), "act_fwd")
    return y


def act_bwd(y, dy, act: int, slope=0.01):
    if not y.is_cuda:
        return ref.act_bwd(y, dy, act, slope)
    dx = torch.empty_like(dy)
    check(_k("ddl_act_bwd", y)(ptr(y), ptr(dy), ptr(dx), y.numel(), act, float(slope),
                                     stream()), "act_bwd")
    return dx


def channel_sum(x, out):
    """out[G, C] (view, fp32) += sum over all but first/last dims of x."""
    if F32.is_f32(x):
        return F32.channel_sum(x.contiguous(), out)
    if not x.is_cuda:
        ref.channel_sum(x, out)
        return out
    G, C = x.shape[0], x.shape[-1]
    check(_k("ddl_channel_sum", x)(ptr(x), ptr(out), _gs(out), x[0].numel() // C, C, G,
                                         stream()), "channel_sum")
    return out


def gemm_nt_bf16(x, w, out=None):
    """y[T][V] = x[T][C] . w[V][C]^T, bf16 in / out, fp32 accumulate (csrc/kernels/gemm_bf16.hip:
    the wide-output LM-head GEMM, C % 32 == 0, V % 8 == 0)."""
    T, C = x.shape
    V = w.shape[0]
    if not x.is_cuda:
        return (x.float() @ w.float().t()).to(x.dtype)
    assert x.dtype == w.dtype == torch.bfloat16 and x.is_contiguous() and w.is_contiguous()
    assert w.shape[1] == C
    if out is None:
        out = torch.empty(T, V, dtype=torch.bfloat16, device=x.device)
    check(_lib.kernels().ddl_gemm_nt_bf16(ptr(x), ptr(w), ptr(out), T, V, C, out.stride(0), stream()),
          "gemm_nt_bf16")
    return out


def gemm_nt_ok(C: int, V: int) -> bool:
    return C % 32 == 0 and C >= 32 and V % 8 == 0


def to_bf16(x32: torch.Tensor, out=None):
    out = out if out is not None else torch.empty(x32.shape, dtype=torch.bfloat16, device=x32.device)
    if not x32.is_cuda:
        out.copy_(x32)
        return out
    assert x32.is_contiguous() and out.is_contiguous()
    check(_lib.kernels().ddl_cast_f32_bf16(ptr(x32), ptr(out), x32.numel(), stream()), "cast")
    return out


def _im2col_k(im2col) -> int:
    return 3 if im2col is True else int(im2col or 0)


def _stem_out(H, W, k, pad, stride):
    if not k:
        return H, W
    return (H + 2 * pad - k) // stride + 1, (W + 2 * pad - k) // stride + 1


def _im2col_cpu(xf, k, pad, stride, cpad, dtype=torch.bfloat16):
    N, C, H, W = xf.shape
    Ho, Wo = _stem_out(H, W, k, pad, stride)
    if k:
        cols = torch.nn.functional.unfold(xf, k, padding=pad, stride=stride)  # [N, C*k*k, L]
        cols = cols.reshape(N, C, k * k, Ho * Wo).permute(0, 3, 2, 1).reshape(N, Ho, Wo, k * k * C)
    else:
        cols = xf.permute(0, 2, 3, 1)
    out = torch.zeros(1, N, Ho, Wo, cpad, dtype=torch.float32)
    out[0, ..., :cols.shape[-1]] = cols
    return out if dtype == torch.float32 else ref._bf(out)


def nchw_to_nhwc(x: torch.Tensor, cpad: int, im2col=0, pad: int = 0, stride: int = 1,
                 dtype=torch.bfloat16):
    """fp32 NCHW -> NHWC [1, N, H', W', cpad] (bf16, or fp32 for the reference-precision mode);
    ``im2col=k`` lays out the k x k / stride patches of the stem conv as channels
    ((r*k+s)*C + c), so the stem runs as a 1x1 GEMM."""
    k = _im2col_k(im2col)
    N, C, H, W = x.shape
    Ho, Wo = _stem_out(H, W, k, pad, stride)
    if not x.is_cuda:
        return _im2col_cpu(x.float(), k, pad, stride, cpad, dtype)
    xc = x.float().contiguous()
    out = torch.empty(1, N, Ho, Wo, cpad, dtype=dtype, device=x.device)
    check(_k("ddl_nchw_to_nhwc", out)(ptr(xc), ptr(out), N, C, H, W, cpad, k, pad, stride,
                                          stream()), "nchw_to_nhwc")
    return out


def prep_images(src_u8, idx, mean, inv_std, cpad, im2col=0, pad=0, stride=1, out=None,
                labels=None, labels_out=None, dtype=torch.bfloat16):
    """Gather uint8 HWC samples by id, normalise, NHWC bf16 / fp32 (``dtype``; channel-padded /
    stem-im2col). labels / labels_out: also gather the int32 labels of the batch (same launch)."""
    k = _im2col_k(im2col)
    n = idx.numel()
    Hs, Ws, Cs = src_u8.shape[1:]
    Ho, Wo = _stem_out(Hs, Ws, k, pad, stride)
    if out is None:
        out = torch.empty(n, Ho, Wo, cpad, dtype=dtype, device=src_u8.device)
    if not src_u8.is_cuda:
        ids = idx.long().reshape(-1)
        x = src_u8[ids].float() / 255.0
        x = (x - mean) * inv_std
        out.copy_(_im2col_cpu(x.permute(0, 3, 1, 2), k, pad, stride, cpad, out.dtype)[0].reshape(out.shape))
        if labels is not None:
            labels_out.copy_(labels[ids].reshape(labels_out.shape))
        return out
    assert idx.dtype == torch.int32 and idx.is_contiguous()
    assert labels is None or (labels.dtype == torch.int32 and labels_out.dtype == torch.int32
                              and labels_out.numel() == n)
    check(_k("ddl_prep_images", out)(ptr(src_u8), ptr(idx), ptr(mean), ptr(inv_std), ptr(out),
                                         n, Hs, Ws, Cs, cpad, k, pad, stride, ptr(labels),
                                         ptr(labels_out), stream()),
          "prep_images")
    return out


def maxpool_fwd(x, k, stride, pad, want_argmax=False):
    """-> y, or (y, argmax) with the window-local uint8 argmax that makes the backward a gather."""
    G, N, H, W, C = x.shape
    Ho, Wo = (H + 2 * pad - k) // stride + 1, (W + 2 * pad - k) // stride + 1
    if not x.is_cuda:
        xi = x.float().reshape(G * N, H, W, C).permute(0, 3, 1, 2)
        y = torch.nn.functional.max_pool2d(xi, k, stride, pad)
        y = y.permute(0, 2, 3, 1).reshape(G, N, Ho, Wo, C).to(x.dtype).contiguous()
        return (y, None) if want_argmax else y
    y = torch.empty(G, N, Ho, Wo, C, dtype=x.dtype, device=x.device)
    am = torch.empty(G, N, Ho, Wo, C, dtype=torch.uint8, device=x.device) if want_argmax else None
    check(_k("ddl_maxpool_fwd", x)(ptr(x), ptr(y), ptr(am), G * N, H, W, C, k, stride, pad,
                                         stream()), "maxpool_fwd")
    return (y, am) if want_argmax else y


def maxpool_bwd(x, dy, k, stride, pad, argmax=None):
    G, N, H, W, C = x.shape
    if not x.is_cuda:
        with torch.enable_grad():
            xi = x.float().reshape(G * N, H, W, C).permute(0, 3, 1, 2).detach().requires_grad_(True)
            y = torch.nn.functional.max_pool2d(xi, k, stride, pad)
            g = dy.float().reshape(G * N, *dy.shape[2:]).permute(0, 3, 1, 2)
            (dx,) = torch.autograd.grad(y, xi, g)
        return dx.permute(0, 2, 3, 1).reshape(G, N, H, W, C).to(x.dtype).contiguous()
    dx = torch.empty_like(x)
    check(_k("ddl_maxpool_bwd", x)(ptr(x), ptr(dy), ptr(argmax), ptr(dx), G * N, H, W, C, k,
                                         stride, pad, stream()), "maxpool_bwd")
    return dx


# ------------------------------------------------------------------------------------- loss
def cross_entropy(logits, labels=None, targets=None, ncls=None, scale=1.0, want_grad=True,
                  with_correct=False):
    """Fused softmax-CE over logits [G, N, ld] -> (loss[G] fp32, dlogits bf16|None, correct[G]|None)."""
    G, N, ld = logits.shape
    ncls = ncls or ld
    dev = logits.device
    loss = ws.zeros((G,), dev)
    correct = torch.zeros(G, dtype=torch.int32, device=dev) if with_correct else None
    if not logits.is_cuda:
        d = ref.ce_fwd_bwd(logits, labels, targets, ncls, scale, loss, correct, want_grad)
        return loss, d, correct
    d = torch.empty_like(logits) if want_grad else None
    lab = labels.to(torch.int32).contiguous() if labels is not None else None
    tgt = targets.float().contiguous() if targets is not None else None
    check(_k("ddl_ce_fwd_bwd", logits)(ptr(logits), ptr(lab), ptr(tgt), G * N, N, ncls, ld,
                                        float(scale), ptr(loss), ptr(d), ptr(correct), stream()),
          "ce_fwd_bwd")
    return loss, d, correct


HEAD_FUSED = __import__("os").environ.get("DDL_FUSED_HEAD", "1") != "0"


def head_train_ok(C: int, ncls: int, dtype=torch.bfloat16) -> bool:
    """Shapes the fused classifier head (``head_train``) takes: 8-channel chunks that tile a
    256-thread block, at most 64 classes (one lane per class), class rows of W that fit 32 KiB
    of LDS (fp32 activations: ``functional_f32.head_train_ok``)."""
    if dtype == torch.float32:
        return F32.head_train_ok(C, ncls)
    return C % 8 == 0 and 256 % (C // 8) == 0 and 1 <= ncls <= 64 and ncls * C * 2 <= 32 * 1024


def head_train(x, w, b, labels, ncls: int, scale: float, dw, db, bn=None, with_correct=False):
    """Training step of a classifier head in two launches (loss.hip ``ddl_head_train``): global
    average pool of x [G, N, H, W, C] -> logits = pooled @ w[:, :ncls]^T + b -> softmax CE with hard labels [G, N] (loss[G] =
    scale * sum of the rows' CE) -> dw (+)= dlogits^T @ pooled, db (+)= sum dlogits -> dx = the
    pool's input gradient. w: [G, Kp, (1, 1,) C] bf16 (group-strided view), b: [G, Kp] fp32 or
    None, dw / db: fp32 gradient views of the same shapes. bn = (c, mean, rstd) of the BatchNorm
    whose relu output x is: dx is masked by (x > 0) and the BN's backward sums come back as part
    (as ``avgpool_bwd_bn``). -> (loss[G], correct[G] | None, dx bf16, part | None)."""
    if F32.is_f32(x):
        return F32.head_train(x, w, b, labels, ncls, scale, dw, db, bn=bn, with_correct=with_correct)
    G, N, H, W, C = x.shape
    HW = H * W
    Kp = w.shape[1]
    dev = x.device
    assert ncls <= Kp and head_train_ok(C, ncls), (C, ncls, Kp)
    if not x.is_cuda:
        w2 = w.reshape(G, Kp, C).float()
        pooled = x.float().reshape(G, N, HW, C).mean(2)
        z = torch.einsum("gnc,gkc->gnk", pooled, w2[:, :ncls])
        if b is not None:
            z = z + b.reshape(G, Kp)[:, None, :ncls].float()
        lse = torch.logsumexp(z, -1)
        lab = labels.long().reshape(G, N)
        loss = scale * (lse - z.gather(-1, lab[..., None])[..., 0]).sum(1)
        correct = (z.argmax(-1) == lab).sum(1).to(torch.int32) if with_correct else None
        dl = scale * (torch.softmax(z, -1) - torch.nn.functional.one_hot(lab, ncls).float())
        dw.reshape(G, Kp, C)[:, :ncls] += torch.einsum("gnk,gnc->gkc", dl, pooled)
        if b is not None:
            db.reshape(G, Kp)[:, :ncls] += dl.sum(1)
        dp = torch.einsum("gnk,gkc->gnc", dl, w2[:, :ncls]) / HW
        if bn is None:
            dx = dp[:, :, None, None, :].expand(G, N, H, W, C).to(x.dtype).contiguous()
            return loss, correct, dx, None
        dx, part = _head_pool_bwd_bn_ref(dp, x, bn)
        return loss, correct, dx, part
    assert x.is_contiguous() and labels.is_contiguous()
    loss = ws.zeros((G,), dev)
    correct = torch.zeros(G, dtype=torch.int32, device=dev) if with_correct else None
    dx = torch.empty_like(x)
    a = _lib.HeadArgs()
    a.x, a.w, a.b, a.labels = ptr(x), ptr(w), ptr(b), ptr(labels)
    a.loss, a.correct, a.dw, a.db, a.dx = ptr(loss), ptr(correct), ptr(dw), ptr(db), ptr(dx)
    a.w_gs, a.dw_gs = _gs(w), _gs(dw)
    a.b_gs, a.db_gs = (_gs(b), _gs(db)) if b is not None else (0, 0)
    part = None
    if bn is not None:
        c, mean, rstd = bn
        assert c.is_contiguous() and mean.is_contiguous() and rstd.is_contiguous()
        part = ws.zeros((G, BN_STRIPES, 2, C), dev)
        a.c, a.mean, a.rstd, a.part = ptr(c), ptr(mean), ptr(rstd), ptr(part)
    pooled = torch.empty(G, N, C, dtype=torch.float32, device=dev)
    dlog = torch.empty(G, N, 64, dtype=torch.float32, device=dev)
    a.pooled, a.dlog = ptr(pooled), ptr(dlog)
    a.G, a.N, a.HW, a.C, a.ncls, a.scale = G, N, HW, C, ncls, float(scale)
    check(_lib.kernels().ddl_head_train(ctypes.byref(a), stream()), "head_train")
    return loss, correct, dx, part


def _head_pool_bwd_bn_ref(dp, x, bn):
    """fp32 reference of the head's pool backward with the BN mask and reduce (as avgpool_bwd_bn,
    from an fp32 pooled gradient already divided by HW)."""
    c, mean, rstd = bn
    G, N, H, W, C = x.shape
    d = dp.reshape(G, N, 1, 1, C) * (x.float() > 0)
    dx = d.to(x.dtype).contiguous()
    xh = (c.float() - mean.reshape(G, 1, 1, 1, C)) * rstd.reshape(G, 1, 1, 1, C)
    part = torch.zeros(G, BN_STRIPES, 2, C)
    df = dx.float()
    part[:, 0, 0] = df.reshape(G, -1, C).sum(1)
    part[:, 0, 1] = (df * xh).reshape(G, -1, C).sum(1)
    return dx, part


# --------------------------------------------------------------------------------- optimizers
def sgd_step(p, g, mom, shadow, lr, wd=0.0, momentum=0.0, dampening=0.0, nesterov=False,
             first_step=False, grad_scale=1.0):
    if not p.is_cuda:
        ref.sgd(p, g, mom, shadow, lr, wd, momentum, dampening, nesterov, first_step, grad_scale)
        return
    a = _lib.SGDArgs()
    a.p, a.g, a.mom, a.shadow = ptr(p), ptr(g), ptr(mom), ptr(shadow)
    a.n = p.numel()
    a.lr, a.wd, a.momentum, a.dampening, a.grad_scale = lr, wd, momentum, dampening, grad_scale
    a.nesterov, a.first_step = int(nesterov), int(first_step)
    check(_lib.kernels().ddl_sgd(ctypes.byref(a), stream()), "sgd")


def sgd_direct_step(p, g, shadow, dmap, lr: float, grad_scale: float = 1.0):
    """Finish a direct-SGD step over rows p/g/shadow [rows, P]: the columns ``dmap`` (uint8 per
    16 columns) marks — conv / Linear weights, already stepped by the scaled WGRAD — only refresh
    the bf16 shadow; the others take ``p -= lr * grad_scale * g`` and get their gradient zeroed.
    One launch."""
    if not p.is_cuda:
        ref.sgd_direct(p, g, shadow, dmap, lr, grad_scale)
        return
    assert p.dim() == 2 and p.is_contiguous() and g.is_contiguous()
    assert shadow is None or (shadow.is_contiguous() and shadow.shape == p.shape)
    assert p.shape == g.shape and p.shape[1] % 16 == 0
    assert dmap.dtype == torch.uint8 and dmap.numel() == p.shape[1] // 16 and dmap.is_cuda
    a = _lib.SGDDirectArgs()
    a.p, a.g, a.shadow, a.dmap = ptr(p), ptr(g), ptr(shadow), ptr(dmap)
    a.rows, a.P = p.shape[0], p.shape[1]
    a.lr, a.grad_scale = lr, grad_scale
    check(_lib.kernels().ddl_sgd_direct(ctypes.byref(a), stream()), "sgd_direct")


def adam_step(p, g, m, v, shadow, lr, beta1, beta2, eps, wd, step, decoupled, grad_scale=1.0,
              step_dev=None, row_len: int = 0):
    """One fused Adam/AdamW pass over flat buffers. ``step_dev`` (int64 [1] on the device, already
    advanced to this step) makes the bias correction device-side (HIP-graph capturable).
    ``row_len`` > 0: the buffers are rows of that many elements with one step counter each
    (``step_dev`` [rows]; ``step`` is then a per-row host list on the CPU path)."""
    if not p.is_cuda:
        if row_len > 0:
            for r, t in enumerate(step):
                sl = slice(r * row_len, (r + 1) * row_len)
                ref.adam(p[sl], g[sl], m[sl], v[sl], None if shadow is None else shadow[sl], lr, beta1, beta2,
                         eps, wd, t, decoupled, grad_scale)
            return
        ref.adam(p, g, m, v, shadow, lr, beta1, beta2, eps, wd, step, decoupled, grad_scale)
        return
    a = _lib.AdamArgs()
    a.p, a.g, a.m, a.v, a.shadow = ptr(p), ptr(g), ptr(m), ptr(v), ptr(shadow)
    a.n = p.numel()
    a.lr, a.beta1, a.beta2, a.eps, a.wd, a.grad_scale = lr, beta1, beta2, eps, wd, grad_scale
    if row_len > 0:  # per-row device step counters: the kernel computes the corrections
        a.bc1 = a.bc2 = 1.0
        assert step_dev is not None and step_dev.numel() * row_len == p.numel()
    else:
        a.bc1, a.bc2 = 1 - beta1 ** step, 1 - beta2 ** step
    a.decoupled = int(decoupled)
    a.step_dev = ptr(step_dev)
    a.row_len = int(row_len)
    check(_lib.kernels().ddl_adam(ctypes.byref(a), stream()), "adam")


def bce_logits(logits, target, scale=1.0, want_grad=True):
    """Binary CE on column 0 of logits [R, ld] (bf16 or fp32). target: float or fp32 [R] tensor.
    -> (loss_sum fp32 [1], dlogits [R, ld] (logits' dtype) with (sigmoid(l)-t)*scale in column 0, or None)."""
    R, ld = logits.shape
    if not logits.is_cuda:
        t = target if torch.is_tensor(target) else torch.full((R,), float(target))
        loss, d = ref.bce_logits(logits[:, 0].float(), t.float())
        dl = None
        if want_grad:
            dl = torch.zeros_like(logits)
            dl[:, 0] = (d * scale).to(logits.dtype)
        return loss.reshape(1), dl
    if logits.dtype == torch.float32:  # deterministic fp32 kernel (one workgroup, fixed-order sum)
        assert logits.is_contiguous()
        loss = torch.empty(1, dtype=torch.float32, device=logits.device)
        dl = torch.empty_like(logits) if want_grad else None  # every element written by the kernel
        tt = target.float().contiguous() if torch.is_tensor(target) else None
        check(_lib.kernels().ddl_bce_logits_f32(ptr(logits), ld, ptr(tt), 0.0 if tt is not None else float(target), R,
                                                float(scale), ptr(loss), ptr(dl), stream()), "bce_logits_f32")
        return loss, dl
    assert logits.is_contiguous() and logits.dtype == torch.bfloat16
    loss = torch.zeros(1, dtype=torch.float32, device=logits.device)
    dl = torch.zeros_like(logits) if want_grad else None
    tt = target.float().contiguous() if torch.is_tensor(target) else None
    tv = 0.0 if tt is not None else float(target)
    check(_lib.kernels().ddl_bce_logits(ptr(logits), ld, ptr(tt), tv, R, float(scale), ptr(loss), ptr(dl),
                                        stream()), "bce_logits")
    return loss, dl


def gan_inputs(desc, steps: int, B: int, nz: int, idx_out, z_out):
    """Federated-GAN round inputs (batch indices + generator noise) for G slots, each a pure
    function of its client's seed: ``desc`` [(seed, n, off), ...] (host list) or a device int64
    [G, 3] tensor; writes idx_out [steps, G*B] int64 and z_out [steps, G, B, nz] fp32 (nn_ops.hip
    gan_inputs_kernel; on CPU tensors the numpy twin ``reference.gan_inputs``)."""
    if not idx_out.is_cuda:
        idx, z = ref.gan_inputs(desc, steps, B, nz)
        idx_out.copy_(idx.view_as(idx_out))
        z_out.copy_(z.view_as(z_out))
        return idx_out, z_out
    if not torch.is_tensor(desc):
        desc = torch.tensor(desc, dtype=torch.int64).pin_memory().to(idx_out.device, non_blocking=True)
    G = desc.shape[0]
    assert idx_out.is_contiguous() and z_out.is_contiguous() and idx_out.dtype == torch.int64
    assert idx_out.numel() == steps * G * B and z_out.numel() == steps * G * B * nz
    check(_lib.kernels().ddl_gan_inputs(ptr(desc), G, steps, B, nz, ptr(idx_out), ptr(z_out), stream()),
          "gan_inputs")
    return idx_out, z_out


# ------------------------------------------------------------------------------- aggregation
def weighted_sum(src, coeff, out, accumulate=False):
    """out[P] (+)= sum_g coeff[g] * src[g, :P] (src rows may be strided views of a [G, *] buffer)."""
    if not src.is_cuda:
        ref.weighted_sum(src, coeff, out, accumulate)
        return out
    assert src.stride(1) == 1 and out.is_contiguous()
    check(_lib.kernels().ddl_weighted_sum(ptr(src), src.stride(0), ptr(coeff.float().contiguous()),
                                          src.shape[0], out.numel(), ptr(out), int(accumulate),
                                          stream()), "weighted_sum")
    return out


def broadcast_rows(src, dst, shadow=None):
    if not src.is_cuda:
        ref.broadcast_rows(src, dst, shadow)
        return
    assert dst.stride(1) == 1
    check(_lib.kernels().ddl_broadcast_rows(ptr(src), ptr(dst), dst.stride(0), dst.shape[0],
                                            src.numel(), ptr(shadow),
                                            0 if shadow is None else shadow.stride(0), stream()),
          "broadcast_rows")


MAX_ROBUST_CLIENTS = 128  # K limit of the native Gram / coordinate-selection kernels


def _robust_k(K, what):
    if not 1 <= K <= MAX_ROBUST_CLIENTS:
        raise ValueError(f"{what}: K={K} client rows; the native kernel takes 1..{MAX_ROBUST_CLIENTS} "
                         "(shard the clients over more GPUs, or pre-aggregate buckets of clients)")


def gram(X, center=None):
    """(X - c)(X - c)^T for X [K, n] fp32 (K <= 128) on the exact-fp32 MFMA; per-block partial
    Grams summed in a fixed order, so the result is bit-reproducible."""
    if not X.is_cuda:
        return ref.gram(X, center)
    K, n = X.shape
    if K > MAX_ROBUST_CLIENTS:
        return _gram_blocked(X, center)
    _robust_k(K, "gram")
    assert X.dtype == torch.float32 and X.stride(1) == 1
    out = torch.empty(K, K, dtype=torch.float32, device=X.device)
    cap = _lib.kernels().ddl_gram_f32_workspace(K, n)
    part = torch.empty(max(cap, 1), dtype=torch.float32, device=X.device)
    check(_lib.kernels().ddl_gram_f32(ptr(X), X.stride(0), ptr(center), K, n, ptr(part), cap, ptr(out),
                                      stream()), "gram_f32")
    out._keep = part  # the scratch must outlive the (asynchronous) launches
    return out


def _gram_blocked(X, center=None):
    """Gram of K > MAX_ROBUST_CLIENTS rows: the native Gram of every pair of row blocks stacked
    ([A; B], <= MAX_ROBUST_CLIENTS rows) yields A A^T, A B^T and B B^T; each output block comes from
    one fixed-order native reduction, so the result stays bit-reproducible."""
    K = X.shape[0]
    bs = MAX_ROBUST_CLIENTS // 2
    nb = -(-K // bs)
    out = torch.empty(K, K, dtype=torch.float32, device=X.device)
    for i in range(nb):
        a0, a1 = i * bs, min(K, (i + 1) * bs)
        for j in range(i, nb):
            b0, b1 = j * bs, min(K, (j + 1) * bs)
            if i == j:
                out[a0:a1, a0:a1] = gram(X[a0:a1].contiguous(), center)
                continue
            gp = gram(torch.cat([X[a0:a1], X[b0:b1]]), center)
            na = a1 - a0
            out[a0:a1, b0:b1] = gp[:na, na:]
            out[b0:b1, a0:a1] = gp[na:, :na]
    return out


def pack_shards(rows, W: int, S: int, gmax: int, out=None):
    """The coordinate-sharded aggregators' all-to-all send buffer in one pass: out[w][g][s] =
    rows[g][w*S + s] (zero past P and for g >= G). rows [G, P] with unit column stride."""
    G, P = rows.shape
    if out is None:
        out = torch.empty(W, gmax, S, dtype=torch.float32, device=rows.device)
    if not rows.is_cuda:
        out.zero_()
        if G:
            pad = torch.zeros(G, W * S, dtype=torch.float32)
            pad[:, :P] = rows
            out[:, :G] = pad.reshape(G, W, S).transpose(0, 1)
        return out
    assert rows.dtype == torch.float32 and (G == 0 or rows.stride(1) == 1) and out.is_contiguous()
    check(_lib.kernels().ddl_pack_shards(ptr(rows) if G else ptr(out), rows.stride(0) if G else 0, G, P, W, S,
                                         gmax, ptr(out), stream()), "pack_shards")
    return out


def krum_select(gram, nb: int, m: int, keys=None):
    """Krum scores (sum of the nb smallest squared distances to the other clients) from a K x K Gram,
    and the m clients of least score -> (scores [K] fp32, sel [m] int32 row indices). Exact ties go
    to the smaller key (``keys``: a per-row int list, default the row index)."""
    K = gram.shape[0]
    if keys is None:
        keys = list(range(K))
    if not gram.is_cuda:
        sq = torch.diagonal(gram)
        d2 = (sq[:, None] + sq[None, :] - 2 * gram).clamp_min(0)
        d2.fill_diagonal_(float("inf"))
        scores = torch.sort(d2, 1).values[:, :nb].sum(1)
        order = sorted(range(K), key=lambda i: (float(scores[i]), keys[i]))
        return scores, torch.tensor(order[:m], dtype=torch.int32)
    assert gram.dtype == torch.float32 and gram.is_contiguous() and K <= MAX_ROBUST_CLIENTS
    scores = torch.empty(K, dtype=torch.float32, device=gram.device)
    sel = torch.empty(m, dtype=torch.int32, device=gram.device)
    kt = torch.tensor(keys, dtype=torch.int32).to(gram.device, non_blocking=True)
    check(_lib.kernels().ddl_krum_select(ptr(gram), K, nb, m, ptr(kt), ptr(scores), ptr(sel), stream()),
          "krum_select")
    scores._keep = kt
    return scores, sel


def mean_rows_idx(X, sel, out=None):
    """out = (1/m) sum over the rows X[sel[t]] in selection order (products rounded, then added)."""
    n = X.shape[1]
    m = sel.numel()
    if out is None:
        out = torch.empty(n, dtype=torch.float32, device=X.device)
    if not X.is_cuda:
        rows = X.index_select(0, sel.long())
        out.zero_()
        for t in range(m):
            out.add_(rows[t] * (1.0 / m))
        return out
    assert X.dtype == torch.float32 and X.stride(1) == 1 and sel.dtype == torch.int32
    check(_lib.kernels().ddl_mean_rows_idx(ptr(X), X.stride(0), ptr(sel), m, n, ptr(out), stream()),
          "mean_rows_idx")
    return out


def coord_select(X, mode: str, trim: int = 0):
    """Coordinate-wise median ('median') or trimmed mean ('trimmed') over K rows of X [K, n]."""
    m = 0 if mode == "median" else 1
    if not X.is_cuda:
        return ref.coord_select(X, m, trim)
    _robust_k(X.shape[0], f"coord_select({mode})")
    assert X.dtype == torch.float32 and X.stride(1) == 1
    out = torch.empty(X.shape[1], dtype=torch.float32, device=X.device)
    check(_lib.kernels().ddl_coord_select(ptr(X), X.stride(0), X.shape[0], X.shape[1], m, trim,
                                          ptr(out), stream()), "coord_select")
    return out
