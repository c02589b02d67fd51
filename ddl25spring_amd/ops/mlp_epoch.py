"""A whole training epoch of a small fp32 MLP graph in ONE kernel launch (csrc/kernels/mlp_epoch.hip).

The vertical-FL split-NN (reference lab/tutorial_2b/vfl.py:11-102: per-party ``BottomModel``
Linear-ReLU-Linear-ReLU-Dropout, concat, ``TopModel`` Linear-Leaky x3 + Dropout, soft-target CE,
AdamW, one step per mini-batch) is ~44 K parameters on 64-row mini-batches: unfused, each
mini-batch is ~40 latency-bound launches. ``MlpEpoch`` describes the net as a table of
buffers (activation width / act / dropout) and layers (in -> out column ranges, level), and one
persistent workgroup runs every forward level, the CE, every backward level and the AdamW update
of every mini-batch of the epoch, on exact-fp32 MFMAs.

Numerics: the same math as the module path (fp32 products, FlatAdam's AdamW arithmetic); the
dropout masks come from Philox(seed; element, optimizer step, buffer) rather than torch's
generator. ``reference_epoch`` is the same epoch in torch (CPU, fp32 or float64) with the SAME
masks: the CPU path of ``MlpEpoch`` and the numerics test of the kernel.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass, field

import numpy as np
import torch

from . import _lib
from ._lib import check, ptr, stream

vp, i32, i64, u64, f32 = _lib.vp, _lib.i32, _lib.i64, _lib.u64, _lib.f32
MAXL, MAXB, MAXP, MAXLEV = 12, 12, 4, 8
NPROF = 2 * MAXLEV + 2  # mlp_epoch.hip phase-clock slots
ACTS = {"none": 0, "relu": 1, "leaky_relu": 2}


class MlpBuf(ctypes.Structure):  # mlp_epoch.hip MlpBuf
    _fields_ = [("off", i32), ("ld", i32), ("width", i32), ("act", i32), ("slope", f32), ("drop", f32)]


class MlpLayer(ctypes.Structure):  # mlp_epoch.hip MlpLayer
    _fields_ = [("in_buf", i32), ("in_col", i32), ("out_buf", i32), ("out_col", i32), ("K", i32), ("N", i32),
                ("level", i32), ("need_dx", i32), ("w", i64), ("b", i64)]


class MlpEpochArgs(ctypes.Structure):  # mlp_epoch.hip MlpEpochArgs
    _fields_ = [("x", vp * MAXP), ("x_ld", i32 * MAXP), ("y", vp), ("p", vp), ("g", vp), ("m", vp), ("v", vp),
                ("step_dev", vp), ("stats", vp), ("prof", vp), ("nparam", i64), ("lds_floats", i64),
                ("seed", u64), ("lr", f32), ("beta1", f32), ("beta2", f32), ("eps", f32), ("wd", f32),
                ("n", i32), ("B", i32), ("ncls", i32), ("nlayers", i32), ("nbufs", i32), ("nlev", i32),
                ("logits_buf", i32), ("probe", i32), ("bufs", MlpBuf * MAXB), ("layers", MlpLayer * MAXL)]


_lib.register_signatures({"ddl_mlp_epoch": [ctypes.POINTER(MlpEpochArgs), vp, vp], "ddl_mlp_epoch_args_size": [],
                          "ddl_mlp_epoch_lds_max": []})
LDS_MAX_BYTES = 160 * 1024 - 1024  # mlp_epoch.hip LDS_MAX_BYTES: every activation of a mini-batch lives in LDS
DROP_MAGIC = 0x7F4A7C15  # mlp_epoch.hip drop4(): Philox counter word 2
_VARIANT = os.environ.get("DDL_MLP_LIB", "")  # a standalone build of mlp_epoch.hip (A/B timing)
_vlib = None


def _kern():
    """The library holding ddl_mlp_epoch: the kernel library, or a DDL_MLP_LIB variant build."""
    global _vlib
    if not _VARIANT:
        return _lib.kernels()
    if _vlib is None:
        _lib.kernels()  # torch's HIP runtime first
        _vlib = ctypes.CDLL(_VARIANT)
        _vlib.ddl_mlp_epoch.argtypes = [ctypes.POINTER(MlpEpochArgs), vp, vp]
        _vlib.ddl_mlp_epoch.restype = ctypes.c_int
        _vlib.ddl_mlp_epoch_args_size.restype = ctypes.c_int
    return _vlib


# ------------------------------------------------------------------------------------ graph
@dataclass
class Buf:
    width: int
    act: str = "none"
    slope: float = 0.01
    drop: float = 0.0

    @property
    def ld(self) -> int:
        """Row pitch in the kernel's LDS arena: whole float4s plus one (rows land 4 banks apart)."""
        return -(-self.width // 4) * 4 + 4


@dataclass
class Layer:
    weight: torch.Tensor  # [N][K] parameter
    bias: torch.Tensor    # [N]
    in_buf: int           # >= 0 buffer, < 0 party input -(p + 1)
    in_col: int
    out_buf: int
    out_col: int
    level: int
    need_dx: bool = True

    @property
    def N(self) -> int:
        return self.weight.shape[0]

    @property
    def K(self) -> int:
        return self.weight.shape[1]


@dataclass
class Graph:
    bufs: list[Buf] = field(default_factory=list)
    layers: list[Layer] = field(default_factory=list)
    logits_buf: int = -1
    n_inputs: int = 0

    @property
    def nlev(self) -> int:
        return 1 + max(L.level for L in self.layers)

    def validate(self):
        if not (0 < len(self.layers) <= MAXL and 0 < len(self.bufs) <= MAXB and self.nlev <= MAXLEV
                and 0 < self.n_inputs <= MAXP and 0 <= self.logits_buf < len(self.bufs)):
            raise ValueError("MLP graph exceeds the fused epoch kernel's tables")
        seen = set()
        for L in self.layers:
            if L.bias is None:
                raise ValueError("fused MLP epoch: every layer needs a bias")
            if L.out_col + L.N > self.bufs[L.out_buf].width:
                raise ValueError("layer output overruns its buffer")
            if L.in_buf >= 0:
                if L.in_col + L.K > self.bufs[L.in_buf].width:
                    raise ValueError("layer input overruns its buffer")
                if L.need_dx:  # one writer per input gradient column range (no accumulation)
                    key = (L.in_buf, L.in_col)
                    if key in seen:
                        raise ValueError("two layers back-propagate into the same input columns")
                    seen.add(key)
            elif L.need_dx:
                raise ValueError("party inputs take no gradient")


def splitnn_graph(bottoms, top) -> Graph:
    """The split-NN of models/tabular.py (BottomModel per party, TopModel) as an MLP graph."""
    from ..models import tabular as T
    g = Graph(n_inputs=len(bottoms))
    drops, col = set(), 0
    for p, bm in enumerate(bottoms):
        if not isinstance(bm, T.BottomModel):
            raise TypeError("splitnn_graph: bottoms must be tabular.BottomModel")
        g.bufs.append(Buf(bm.fc1.out_features, bm.fc1.act_kind, bm.fc1.slope))
        drops.add((bm.fc2.act_kind, bm.fc2.slope, bm.dropout.p))
    if len(drops) != 1:
        raise ValueError("bottoms differ in cut-layer activation / dropout")
    act, slope, p_drop = drops.pop()
    cut = len(g.bufs)
    g.bufs.append(Buf(top.in_size, act, slope, p_drop))
    for p, bm in enumerate(bottoms):
        g.layers.append(Layer(bm.fc1.weight, bm.fc1.bias, -(p + 1), 0, p, 0, 0, need_dx=False))
        g.layers.append(Layer(bm.fc2.weight, bm.fc2.bias, p, 0, cut, col, 1))
        col += bm.fc2.out_features
    if col != top.in_size:
        raise ValueError("bottom widths do not add up to the top model's input")
    prev = cut
    fcs = [top.fc1, top.fc2, top.fc3]
    for i, fc in enumerate(fcs):
        last = i == len(fcs) - 1
        g.bufs.append(Buf(fc.out_features, fc.act_kind, fc.slope, top.dropout.p if last else 0.0))
        g.layers.append(Layer(fc.weight, fc.bias, prev, 0, len(g.bufs) - 1, 0, 2 + i))
        prev = len(g.bufs) - 1
    g.logits_buf = prev
    g.validate()
    return g


# ------------------------------------------------------------------------------------ masks
def keep_mask(seed: int, step: int, buf: int, M: int, ld: int, c0: int, ncols: int, p: float) -> torch.Tensor:
    """mlp_epoch.hip drop4() on the host: keep mask bool [M][ncols] for buffer columns c0 .. c0 + ncols
    (element (p, c): word p & 3 of Philox(seed; (p >> 2) * ld + c, step, DROP_MAGIC, buf) > p)."""
    from . import reference as ref
    m = np.arange(M, dtype=np.int64)[:, None]
    c = np.arange(c0, c0 + ncols, dtype=np.int64)[None, :]
    ctr = ((m >> 2) * ld + c).astype(np.uint32)  # one Philox call per 4 rows of a column
    z = np.zeros_like(ctr)
    r = ref.philox4x32(ctr, z + np.uint32(step & 0xFFFFFFFF), z + np.uint32(DROP_MAGIC),
                       z + np.uint32(buf), seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)
    w = (np.zeros_like(c) + m & 3).astype(np.uint32)
    u = np.where(w == 0, r[0], np.where(w == 1, r[1], np.where(w == 2, r[2], r[3])))
    return torch.from_numpy(ref._unit(u) > np.float32(p))


def _act(v, kind, slope):
    return torch.relu(v) if kind == "relu" else (torch.where(v > 0, v, slope * v) if kind == "leaky_relu" else v)


def _act_grad(z, kind, slope):
    one = torch.ones_like(z)
    if kind == "relu":
        return (z > 0).to(z.dtype)
    if kind == "leaky_relu":
        return torch.where(z > 0, one, torch.full_like(z, slope))
    return one


def reference_epoch(g: Graph, flat: dict, offsets: dict, xs, y, B: int, seed: int, step0: int,
                    lr: float, betas, eps: float, wd: float, dtype=torch.float32):
    """The fused epoch in torch on the CPU: ``flat`` = {"p", "g", "m", "v"} 1-D tensors (updated in
    place), ``offsets[id(param)]`` = its offset. Returns (sum of batch-mean losses, correct)."""
    dt = dtype
    P = {k: v.to(dt) for k, v in flat.items()}
    xs = [x.to(dt) for x in xs]
    y = y.to(dt)
    n = y.shape[0]
    loss_sum, correct = 0.0, 0
    b1, b2 = betas

    def W(L):
        o = offsets[id(L.weight)]
        return P["p"][o:o + L.N * L.K].view(L.N, L.K)

    def bvec(L):
        o = offsets[id(L.bias)]
        return P["p"][o:o + L.N]

    for s, r0 in enumerate(range(0, n, B)):
        M = min(B, n - r0)
        t = step0 + s + 1
        act = [torch.zeros(M, b.ld, dtype=dt) for b in g.bufs]
        dact = [torch.zeros(M, b.ld, dtype=dt) for b in g.bufs]

        def inp(L):
            if L.in_buf < 0:
                return xs[-L.in_buf - 1][r0:r0 + M, L.in_col:L.in_col + L.K]
            return act[L.in_buf][:, L.in_col:L.in_col + L.K]

        def mask(bi, c0, nc):
            b = g.bufs[bi]
            return keep_mask(seed, t, bi, M, b.ld, c0, nc, b.drop)

        for lev in range(g.nlev):
            for L in g.layers:
                if L.level != lev:
                    continue
                ob = g.bufs[L.out_buf]
                v = _act(inp(L) @ W(L).t() + bvec(L), ob.act, ob.slope)
                if ob.drop > 0:
                    v = torch.where(mask(L.out_buf, L.out_col, L.N), v * (1.0 / (1.0 - ob.drop)), torch.zeros_like(v))
                act[L.out_buf][:, L.out_col:L.out_col + L.N] = v
        lb = g.bufs[g.logits_buf]
        C = y.shape[1]
        z = act[g.logits_buf][:, :C]
        tg = y[r0:r0 + M]
        lse = torch.logsumexp(z, 1, keepdim=True)
        ts = tg.sum(1, keepdim=True)
        loss_sum += float((ts * lse - (tg * z).sum(1, keepdim=True)).sum() / M)
        correct += int((z.argmax(1) == tg.argmax(1)).sum())
        d = (torch.softmax(z, 1) * ts - tg) / M * _act_grad(z, lb.act, lb.slope)
        if lb.drop > 0:
            d = torch.where(mask(g.logits_buf, 0, C), d * (1.0 / (1.0 - lb.drop)), torch.zeros_like(d))
        dact[g.logits_buf][:, :C] = d
        for lev in reversed(range(g.nlev)):
            for L in g.layers:
                if L.level != lev:
                    continue
                dp = dact[L.out_buf][:, L.out_col:L.out_col + L.N]
                ow, ob_ = offsets[id(L.weight)], offsets[id(L.bias)]
                P["g"][ow:ow + L.N * L.K] = (dp.t() @ inp(L)).reshape(-1)
                P["g"][ob_:ob_ + L.N] = dp.sum(0)
                if L.need_dx:
                    ib = g.bufs[L.in_buf]
                    dx = (dp @ W(L)) * _act_grad(act[L.in_buf][:, L.in_col:L.in_col + L.K], ib.act, ib.slope)
                    if ib.drop > 0:
                        dx = torch.where(mask(L.in_buf, L.in_col, L.K), dx * (1.0 / (1.0 - ib.drop)), torch.zeros_like(dx))
                    dact[L.in_buf][:, L.in_col:L.in_col + L.K] = dx
        # AdamW (optim.hip adam_kernel, decoupled)
        bc1, bc2 = 1 - b1 ** t, 1 - b2 ** t
        p_, g_ = P["p"], P["g"]
        p_.mul_(1 - lr * wd)
        P["m"].mul_(b1).add_((1 - b1) * g_)
        P["v"].mul_(b2).add_((1 - b2) * g_ * g_)
        p_.sub_(lr / bc1 * P["m"] / (P["v"].sqrt() / (bc2 ** 0.5) + eps))
    for k in flat:
        flat[k].copy_(P[k].to(flat[k].dtype))
    return loss_sum, correct


# ------------------------------------------------------------------------------------ engine
ENABLED = [os.environ.get("DDL_FUSED_MLP", "1") != "0"]
PROBE = [int(os.environ.get("DDL_MLP_PROBE", "0"))]  # timing probes (wrong results): 1 no GEMM loads, 2 no MFMA


class MlpEpoch:
    """One-launch training epochs of ``graph`` with the flat AdamW ``opt`` (optim.FlatAdam,
    decoupled, no bf16 shadow) over mini-batches of ``batch`` rows; gradients are zeroed per
    mini-batch (the overwrite semantics of zero_grad + backward)."""

    def __init__(self, graph: Graph, opt, batch: int, seed: int | None = None):
        from ..optim import FlatAdam
        if not isinstance(opt, FlatAdam) or not opt.decoupled or opt.shadow is not None:
            raise TypeError("MlpEpoch needs a FlatAdam(W) optimizer (decoupled, no bf16 shadow)")
        graph.validate()
        self.g, self.opt, self.B = graph, opt, int(batch)
        self.offsets = {id(p): off for p, off in zip(opt.params, opt.offsets)}
        used = set()
        for L in graph.layers:
            for t in (L.weight, L.bias):
                if id(t) not in self.offsets:
                    raise ValueError("a layer parameter is not in the optimizer's flat buffer")
                used.add(id(t))
        if used != set(self.offsets):
            raise ValueError("the optimizer holds parameters the MLP graph does not train")
        self.seed = int(torch.randint(0, 2 ** 62, (1,)).item()) if seed is None else int(seed)
        self.offs, tot = [], 0
        rows = -(-self.B // 32) * 32  # whole 32-row tiles (the kernel writes pad rows as zeros)
        for b in graph.bufs:
            self.offs.append(tot)
            tot += rows * b.ld
        self.ncls = graph.bufs[graph.logits_buf].width
        tot += self.B * self.ncls  # the staged mini-batch targets end the arena
        self.lds_floats = tot
        if 4 * tot > LDS_MAX_BYTES:
            raise ValueError(f"MLP epoch: a {self.B}-row mini-batch's activations need {4 * tot} B of LDS "
                             f"(> {LDS_MAX_BYTES})")
        self.prof = None  # set to an int64 [NPROF] device tensor to collect per-phase clocks
        self._dev_args = None  # the tables in device memory (the kernel reads them there)
        self._dev_key = None

    def _args(self, xs, y, stats):
        g = self.g
        a = MlpEpochArgs()
        for p, x in enumerate(xs):
            assert x.is_contiguous() and x.dtype == torch.float32
            a.x[p], a.x_ld[p] = ptr(x), x.shape[1]
        assert y.is_contiguous() and y.dtype == torch.float32 and y.shape[0] == xs[0].shape[0]
        a.y = ptr(y)
        o = self.opt
        a.p, a.g, a.m, a.v = ptr(o.data), ptr(o.grad), ptr(o.m), ptr(o.v)
        a.step_dev, a.stats = ptr(o.t_dev), ptr(stats)
        a.prof = ptr(self.prof)
        a.probe = PROBE[0]
        a.nparam, a.lds_floats, a.seed = o.data.numel(), self.lds_floats, self.seed
        a.lr, a.beta1, a.beta2, a.eps, a.wd = o.lr, o.betas[0], o.betas[1], o.eps, o.weight_decay
        if y.shape[1] != self.ncls:
            raise ValueError(f"targets have {y.shape[1]} classes, the logits buffer {self.ncls}")
        a.n, a.B, a.ncls = y.shape[0], self.B, y.shape[1]
        a.nlayers, a.nbufs, a.nlev, a.logits_buf = len(g.layers), len(g.bufs), g.nlev, g.logits_buf
        for i, b in enumerate(g.bufs):
            a.bufs[i] = MlpBuf(self.offs[i], b.ld, b.width, ACTS[b.act], b.slope, b.drop)
        for i, L in enumerate(g.layers):
            a.layers[i] = MlpLayer(L.in_buf, L.in_col, L.out_buf, L.out_col, L.K, L.N, L.level, int(L.need_dx),
                                   self.offsets[id(L.weight)], self.offsets[id(L.bias)])
        return a

    def run(self, xs, y, stats: torch.Tensor) -> None:
        """One epoch over all rows of ``xs`` (per-party [n][f_p]) / ``y`` ([n][ncls] soft targets);
        ``stats`` (fp32 [2]) += (sum of mini-batch mean losses, correct predictions)."""
        o = self.opt
        steps = -(-y.shape[0] // self.B)
        if not o.data.is_cuda:
            flat = {"p": o.data, "g": o.grad, "m": o.m, "v": o.v}
            ls, cor = reference_epoch(self.g, flat, self.offsets, xs, y, self.B, self.seed, o.t,
                                      o.lr, o.betas, o.eps, o.weight_decay)
            o.t += steps
            stats += torch.tensor([ls, float(cor)], dtype=stats.dtype)
            return
        if o.t_dev is None:
            raise RuntimeError("FlatAdam without a device step counter")
        xs = [x if x.is_contiguous() else x.contiguous() for x in xs]
        y = y if y.is_contiguous() else y.contiguous()
        a = self._args(xs, y, stats)
        key = bytes(a)
        if key != self._dev_key:  # upload once per configuration (same tensors -> same bytes)
            host = torch.frombuffer(bytearray(key), dtype=torch.uint8)
            self._dev_args = host.to(o.data.device)
            self._dev_key = key
        check(_kern().ddl_mlp_epoch(ctypes.byref(a), ptr(self._dev_args), stream()), "mlp_epoch")
        o.t += steps  # host mirror of the device counter the kernel advanced


def abi_check() -> None:
    f = _kern().ddl_mlp_epoch_args_size
    if f() != ctypes.sizeof(MlpEpochArgs):
        raise RuntimeError(f"ABI mismatch for MlpEpochArgs: C {f()} vs ctypes {ctypes.sizeof(MlpEpochArgs)}")
