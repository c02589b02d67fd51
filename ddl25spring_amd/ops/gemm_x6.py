"""Reference-precision (fp32) GEMM on pre-split bf16 planes (csrc/kernels/gemm_x6.hip).

An fp32 matrix is split ONCE into its X6 planes (``split``: three bf16 matrices h, m, l with
x = h + m + l exactly); ``gemm`` multiplies two plane sets in either orientation of each operand,

    out[q * ldo + p] = alpha * sum_k A(p, k) * B(q, k) (+ residual | + old out) (+ bias[p])

with A(p, k) = A[p][k] (K-major) or A[k][p] (MN-major, ``a_mn``), and the same for B. Every product
is exact to one fp32 rounding (six bf16 piece products per fp32 product) and the result is
deterministic (split-K slices folded in slice order). This is the GEMM behind the fp32 LLaMA
linears (ops/llama_f32.py), which run FWD, DGRAD and WGRAD off the same three plane sets:

    y  [T][N] = x [T][K] W^T   : A = W  (K-major), B = x  (K-major)
    dx [T][K] = dy[T][N] W     : A = W  (MN-major), B = dy (K-major)
    dW [N][K] = dy^T x         : A = x  (MN-major), B = dy (MN-major)

On CPU tensors ``split`` keeps the fp32 matrix and ``gemm`` runs the torch fp32 product (tests).
"""
from __future__ import annotations

import ctypes
import os

import torch

from . import _lib
from ._lib import check, ptr, stream

vp, i32, i64, f32 = _lib.vp, _lib.i32, _lib.i64, _lib.f32


class GemmX6Args(ctypes.Structure):  # csrc/kernels/gemm_x6.hip GemmX6Args
    _fields_ = [("a", vp), ("b", vp), ("out", vp), ("res", vp), ("bias", vp), ("partial", vp),
                ("a_ps", i64), ("b_ps", i64), ("partial_cap", i64),
                ("lda", i32), ("ldb", i32), ("ldo", i32), ("M", i32), ("N", i32), ("K", i32),
                ("split_k", i32), ("accumulate", i32), ("alpha", f32), ("probe", i32)]


_lib.register_signatures({
    "ddl_gemm_x6": [vp, i32, vp],
    "ddl_x6_planes": [vp, i64, vp, i64, i64, i32, i32, i32, i32, vp],
    "ddl_gemm_x6_args_size": [],
})


PAD = 32  # planes are zero-padded to whole 32-deep GEMM stages in both dimensions
MAX_PLANE_BYTES = 1 << 30  # 3 planes of one matrix (gemm_x6.hip's 32-bit offsets with out-of-range margins)


def _pad(n: int) -> int:
    return -(-n // PAD) * PAD


class Planes:
    """X6 planes of an fp32 matrix [R][C]: ``data`` int16 [3, Rp, Cp] (bf16 bit patterns h | m | l,
    zero-padded to multiples of 32); on CPU ``data`` is the fp32 matrix itself."""
    __slots__ = ("data", "R", "C")

    def __init__(self, data: torch.Tensor, R: int, C: int):
        self.data, self.R, self.C = data, R, C

    @property
    def is_cuda(self) -> bool:
        return self.data.is_cuda

    @property
    def ld(self) -> int:
        return self.data.shape[-1]

    @property
    def plane_stride(self) -> int:
        return self.data.shape[-1] * self.data.shape[-2]

    def dense(self) -> torch.Tensor:
        """The fp32 matrix back (h + m + l; exact)."""
        if not self.data.is_cuda:
            return self.data
        u = self.data.view(torch.int16).to(torch.int32) & 0xFFFF
        f = (u << 16).view(torch.float32)
        return ((f[2] + f[1]) + f[0])[:self.R, :self.C]


def fits(R: int, C: int) -> bool:
    """Can an [R][C] matrix be a planes-GEMM operand (C % 8, padded planes < MAX_PLANE_BYTES)?"""
    return C % 8 == 0 and 6 * _pad(R) * _pad(C) < MAX_PLANE_BYTES


def split(x: torch.Tensor, out: torch.Tensor | None = None) -> Planes:
    """The X6 planes of a 2-D fp32 matrix (rows contiguous, C % 8 == 0 on the device)."""
    assert x.dim() == 2
    R, C = x.shape
    if not x.is_cuda:
        return Planes(x.float(), R, C)
    if x.dtype != torch.float32:
        raise TypeError("X6 planes split fp32 matrices")
    if x.stride(1) != 1:
        x = x.contiguous()
    Rp, Cp = _pad(R), _pad(C)
    if out is None:
        out = torch.empty(3, Rp, Cp, dtype=torch.int16, device=x.device)
    check(_lib.kernels().ddl_x6_planes(ptr(x), x.stride(0), ptr(out), Cp, Rp * Cp, R, C, Rp, Cp, stream()),
          "x6_planes")
    return Planes(out, R, C)


# ------------------------------------------------------------------------------------ plans
# cfg = TP | TQ << 4 | a_mn << 8 | b_mn << 9 | NS << 12 : block tile (32 TP) x (32 TQ), NS-stage ring
TARGET_WG = int(os.environ.get("DDL_X6G_TARGET_WG", "256"))
_NS = int(os.environ.get("DDL_X6G_NS", "0"))  # LDS ring depth (0: 3 for 128-wide B tiles, else 4)
_FORCE = os.environ.get("DDL_X6G_PLAN", "")  # "TP,TQ,NS,split" (A/B timing)
PROBE = [int(os.environ.get("DDL_X6G_PROBE", "0"))]  # timing probes (wrong results), gemm_x6.hip
_PLANS: dict = {}


def plan(M: int, N: int, K: int) -> tuple[int, int, int, int]:
    """(TP, TQ, NS, split): 96-row tiles where M is a multiple of 96 up to 384 (the 288-wide d_model
    of the tutorial LLaMA: no wasted quarter tile), else 128 x 128; split-K over 32-deep stages until
    ~TARGET_WG workgroups, each slice keeping >= 8 stages."""
    key = (M, N, K)
    p = _PLANS.get(key)
    if p is not None:
        return p
    if _FORCE:
        tp, tq, ns, sp = (int(v) for v in _FORCE.split(","))
        p = (tp, tq, ns, sp)
    elif _tuned_plan(M, N, K) is not None:
        p = _tuned_plan(M, N, K)
    else:
        tp = 3 if (M % 96 == 0 and M <= 384) else 4
        tq = 4
        tiles = -(-M // (32 * tp)) * -(-N // (32 * tq))
        nk = -(-K // 32)
        sp = 1
        while tiles * sp < TARGET_WG and nk >= sp * 2 * 8 and sp < 64:
            sp *= 2
        p = (tp, tq, _NS or (3 if tq == 4 else 4), sp)
    _PLANS[key] = p
    return p


def _tuned_plan(M: int, N: int, K: int):
    """A measured plan ('x6g:M,N,K' entries of f32_plans.json, scripts/llm_linear_tune_x6g.py)."""
    from . import functional_f32 as F32
    F32._tuned(F32.F_FWD, _GEOM_PROBE)  # loads the table
    v = F32._TUNED.get(f"x6g:{M},{N},{K}")
    return None if v is None else tuple(int(t) for t in v)


class _GeomProbe:  # any geometry: _tuned() only needs one to load the table
    G = N = H = W = C = K = R = S = P = Q = stride = pad = 1


_GEOM_PROBE = _GeomProbe()


def _extent(pl: Planes, mn: bool) -> tuple[int, int]:
    """(output extent, reduction extent) of a plane set read K-major (rows = output) or MN-major."""
    return (pl.C, pl.R) if mn else (pl.R, pl.C)


def gemm(a: Planes, a_mn: bool, b: Planes, b_mn: bool, out: torch.Tensor, *, residual=None, bias=None,
         accumulate: bool = False, alpha: float = 1.0, split_k: int = 0, ws_role: str = "main") -> torch.Tensor:
    """out[q][p] (row pitch out.stride(0)) = alpha * A . B^T (+ residual | + out) (+ bias[p])."""
    M, K = _extent(a, a_mn)
    N, Kb = _extent(b, b_mn)
    if K != Kb:
        raise ValueError(f"X6 GEMM reduction extents differ: {K} vs {Kb}")
    assert out.dim() == 2 and out.shape[0] == N and out.shape[1] >= M and out.stride(1) == 1
    if not a.is_cuda:
        A = a.data.t() if a_mn else a.data
        B = b.data.t() if b_mn else b.data
        prod = (B.double() @ A.double().t()).float() if os.environ.get("DDL_X6G_CPU64") else B @ A.t()
        prod = alpha * prod
        if residual is not None:
            prod = prod + residual
        elif accumulate:
            prod = prod + out[:, :M]
        if bias is not None:
            prod = prod + bias.view(1, M)
        out[:, :M].copy_(prod)
        return out
    tp, tq, ns, sp = plan(M, N, K)
    if split_k:
        sp = split_k
    ar = GemmX6Args()
    ar.a, ar.b, ar.out = ptr(a.data), ptr(b.data), ptr(out)
    ar.res = ptr(residual)
    if residual is not None:
        assert residual.stride() == out.stride()
    ar.bias = ptr(bias)
    ar.a_ps, ar.b_ps = a.plane_stride, b.plane_stride
    ar.lda, ar.ldb, ar.ldo = a.ld, b.ld, out.stride(0)
    ar.M, ar.N, ar.K = M, N, K
    ar.accumulate, ar.alpha = int(bool(accumulate)), float(alpha)
    if sp > 1:
        from .functional_f32 import workspace
        buf = workspace(out.device, ws_role)
        while sp > 1 and sp * M * N > buf.numel():
            sp //= 2
        if sp > 1:
            ar.partial, ar.partial_cap = ptr(buf), buf.numel()
    ar.split_k = sp
    ar.probe = PROBE[0]
    cfg = tp | (tq << 4) | (int(bool(a_mn)) << 8) | (int(bool(b_mn)) << 9) | (ns << 12)
    check(_lib.kernels().ddl_gemm_x6(ctypes.byref(ar), cfg, stream()), "gemm_x6")
    return out
