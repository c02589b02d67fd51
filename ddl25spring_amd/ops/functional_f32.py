"""Reference-precision (fp32) device ops: ctypes front-ends of conv_f32.hip and bn_f32.hip.

``ops.functional`` dispatches here for CUDA tensors of dtype float32 (the fp32 precision mode, see
``models.params.default_precision``); the op signatures and semantics are those of the bf16 ops,
with three differences of representation:
  * BN statistics and BN-backward partial sums are per-tile / per-block *slots* ``[G, S, 2, C]``
    written with plain stores (S depends on the producer's launch), folded in a fixed order — the
    whole fp32 step is deterministic, with no zero-fill launches;
  * a conv's forward statistics buffer is a :class:`SlotStats` holder that the conv fills;
  * ``in_bn=(scale, shift)``: the X operand of FWD / WGRAD is relu(x * scale + shift) computed on
    the fly (operand-side BatchNorm), so a BN+ReLU output that only feeds a conv is never stored.
"""
from __future__ import annotations

import ctypes
import math
import os

import torch

from . import _lib
from . import workspace as ws
from ._lib import check, ptr, stream

F_FWD, F_DGRAD, F_WGRAD = 0, 1, 2
# split-K workspace (floats) per device: partial slices of small-grid FWD / DGRAD / WGRAD
WS_CAP = 1 << 26
_WS: dict = {}
# workgroups a launch should provide before split-K stops (256 CUs, ~2 resident per CU)
TARGET_WG = int(os.environ.get("DDL_F32_TARGET_WG", "640"))


def is_f32(t) -> bool:
    return t is not None and t.is_cuda and t.dtype == torch.float32


class SlotStats:
    """Forward BN statistics of an fp32 conv: ``t`` = [G, slots, 2, C] once the conv has run.
    ``rows`` > 0: slot i holds (sum, M2 about the slot's own mean) of min(rows, M - i*rows)
    output rows (the conv epilogue's per-tile centred statistics, merged exactly in bn_finalize);
    0: (sum, sum of squares) partials (bn_stats)."""
    __slots__ = ("t", "rows")

    def __init__(self):
        self.t = None
        self.rows = 0


def workspace(device, role: str = "main") -> torch.Tensor:
    """The split-K workspace of (device, role): a side-stream WGRAD (role "side",
    functional.wgrad_overlap) runs concurrently with the main stream's split-K launches. Both
    roles are allocated on the first (eager) call; a first call inside a HIP-graph capture raises
    rather than silently dropping to split 1 (which would change the reduction order, so a
    captured step would no longer match the eager one bit for bit)."""
    key = f"{device}:{role}"
    b = _WS.get(key)
    if b is None:
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("fp32 split-K workspace first requested inside a graph capture: run one eager "
                               "step (or functional_f32.ensure_workspace) before capturing")
        ensure_workspace(device)
        b = _WS[key]
    return b


def ensure_workspace(device) -> None:
    for role in ("main", "side"):
        key = f"{device}:{role}"
        if key not in _WS:
            _WS[key] = torch.empty(WS_CAP, dtype=torch.float32, device=device)
            # WGRAD split-K arrival counters (zero between launches: the folding workgroup resets
            # its own), one set per role since the two streams' WGRADs may run concurrently
            _WS[key + ":tickets"] = torch.zeros(TICKETS_CAP, dtype=torch.int32, device=device)
    if torch.device(device).type == "cuda" and _dev_key(device) not in _TICKETS:
        _TICKETS[_dev_key(device)] = torch.zeros(TICKETS_N, dtype=torch.int32, device=device)


# per-(group, phase, tile) counters of the in-kernel split-K fold (the last-arriving slice's
# workgroup sums the slices and runs the epilogue). OFF by default (DDL_F32_WG_FOLD=1 enables it):
# measured 28.5k vs 36.3k samples/s headline and 9.5k vs 21.0k at 1 client — every workgroup's
# device-scope release fence writes back its XCD's L2, and one workgroup folding up to 64 slices
# serially is slower than the parallel reduce launch (profiles/bench_wgfold_r4g.jsonl)
TICKETS_CAP = 1 << 18
WG_FOLD = [os.environ.get("DDL_F32_WG_FOLD", "0") == "1"]


def _dims(mode, g):
    """(Pd, Qd, Kr, phases) of a launch (DGRAD stride 2: the largest phase)."""
    if mode == F_FWD:
        return g.K, g.N * g.P * g.Q, g.R * g.S * g.C, 1
    if mode == F_DGRAD:
        if g.stride == 2:
            hs, wsz = (g.H + 1) // 2, (g.W + 1) // 2
            rn, sn = (g.R + 1) // 2, (g.S + 1) // 2
            return g.C, g.N * hs * wsz, rn * sn * g.K, 4
        return g.C, g.N * g.H * g.W, g.R * g.S * g.K, 1
    return g.K, g.R * g.S * g.C, g.N * g.P * g.Q, 1


def cfg_of(bp: int, bq: int) -> int:
    return (bp // 16) | ((bq // 16) << 8)


# Product engine of the fp32 convolutions (csrc/kernels/conv_f32.hip):
#   "mfma32": exact fp32 MFMA (v_mfma_f32_16x16x4_f32);
#   "x6"    : each fp32 operand split exactly into 3 bf16 pieces, the 6 piece products above one
#             fp32 rounding on the double-rate bf16 MFMA (2.7x fewer MFMA cycles per step);
#   "auto"  : per (mode, geometry) whichever engine the tuner measured faster (plans keyed
#             "auto:...", [bp, bq, split, engine]); untuned launches use X6. Both engines meet the
#             same fp32 tolerances, so mixing them per layer changes only rounding-level detail.
MATHS = ("mfma32", "x6", "auto")
_MATH = [os.environ.get("DDL_F32_MATH", "auto")]
if _MATH[0] not in MATHS:
    raise ValueError(f"DDL_F32_MATH={_MATH[0]!r}: expected one of {MATHS}")


def math() -> str:
    return _MATH[0]


def set_math(name: str) -> None:
    if name not in MATHS:
        raise ValueError(f"fp32 conv math {name!r}: expected one of {MATHS}")
    if name != _MATH[0]:
        _MATH[0] = name
        _PLANS.clear()  # plans are tuned per engine


X6_BIT = 1 << 16
# conv_x6h.hip: the halo-staged X6 kernel (FWD / stride-1 DGRAD of "same" 3x3 and 1x1 convs, 128-pixel
# tiles, pre-split weights). DDL_F32_HALO=0 keeps every launch on conv_f32.hip.
HALO_BIT = 1 << 17
_HALO = [os.environ.get("DDL_F32_HALO", "1") != "0"]
HALO_HPMAX = 288


def set_halo(on: bool) -> None:
    if bool(on) != _HALO[0]:
        _HALO[0] = bool(on)
        _PLANS.clear()


# narrowest image the halo FWD / DGRAD takes by default: 4x4 lost to conv_f32.hip in round 4
# (profiles/x6h_layers_r4.txt) and wins since the round-5 epilogue (c512 at 8 clients, BP 64:
# FWD 406 vs 436 us, DGRAD 417 vs 489, profiles/x6h_l4_r5.txt)
HALO_MIN_W = int(os.environ.get("DDL_F32_HALO_MIN_W", "4"))
# widths that are not a power of two (ResNet-50's 56 / 28) run with rows padded to one
# (DDL_F32_HALO_PADW=0: conv_f32.hip); their tiles are never split over K
HALO_PADW = [os.environ.get("DDL_F32_HALO_PADW", "1") != "0"]


def halo_ok(mode: int, g, auto: bool = False) -> bool:
    """Mirror of conv_x6h.hip x6h_geo: can the halo kernel run this (mode, geometry)? ``auto``: is it
    also the default choice there (explicit plans may pin it where it is not)?"""
    if mode not in (F_FWD, F_DGRAD) or g.stride != 1 or g.R != g.S or g.R not in (1, 3) or g.pad != (g.R - 1) // 2:
        return False
    if g.P != g.H or g.Q != g.W:
        return False
    OH, OWr = g.P, g.Q
    if OWr < 4 or OWr > 128:
        return False
    if auto and OWr < HALO_MIN_W:
        return False
    OW = 1 << (OWr - 1).bit_length()  # rows padded to a power of two (conv_x6h.hip PADW)
    if OW != OWr and (not HALO_PADW[0] or (auto and g.R == 1)):
        # padded 1x1 convs stay on conv_f32.hip's tuned plans by default: a 1x1 conv has no taps
        # to reuse the staged tile (the FLAT1X1 finding, profiles/r50_flat1x1_r4m.txt)
        return False
    TR = 128 // OW
    if TR <= OH:
        if OH % TR:
            return False
        SR = TR
    else:
        if TR % OH:
            return False
        SR = OH
    HP = (TR // SR) * (SR + g.R - 1) * (OW + g.S - 1)
    SC, Pd = (g.C, g.K) if mode == F_FWD else (g.K, g.C)
    if not (HP <= HALO_HPMAX and SC % 16 == 0 and Pd % 4 == 0):
        return False
    return _x6h_native_ok(mode, g)


_X6H_OK: dict = {}


def _x6h_native_ok(mode: int, g) -> bool:
    """The kernel library's own geometry check (x6h_geo: halo layout search, LDS budget) where the
    library is loadable; the Python mirror above only pre-filters, so plan() never picks a halo
    launch that ddl_x6h would refuse."""
    key = (mode, g)
    r = _X6H_OK.get(key)
    if r is None:
        try:
            lib = _lib.kernels()
        except Exception:  # noqa: BLE001 - no library (CPU-only checkout): the mirror decides
            return True
        a = _args(g)
        r = bool(lib.ddl_x6h_ok(ctypes.byref(a), mode, cfg_of(64, 128)))
        _X6H_OK[key] = r
    return r


# A stride-1 1x1 conv is a GEMM over pixels: its image shape does not matter. FLAT1X1 re-shapes
# such a launch as rows of 128 pixels (N = 1, W = 128) whenever N*H*W % 128 == 0 and the image width
# is not already a power of two (ResNet-50's 56 / 28 / 14 / 7), so the halo kernels
# (conv_x6h.hip FWD / DGRAD, conv_x6hw.hip WGRAD) take it; memory layout, strides, BN statistics
# and residual / mask layouts are unchanged. Round 4: ResNet-50 fp32 ran 2.86k vs 3.58k images/s
# with every mode flattened (the image geometry keeps its tuned conv_f32 plans). Round 6, per mode
# (scripts/gpu/r6_flat.sh, images/s): none 3744 / w 3158 / d 3764 / f 3798 / fd 3822 / dw 3240, so
# FWD and DGRAD are flattened by default and WGRAD keeps the image geometry. DDL_F32_FLAT1X1=0 turns
# it off, 1 flattens all modes, or a subset of "fdw".
_FLAT_ENV = os.environ.get("DDL_F32_FLAT1X1", "fd")
FLAT1X1 = [_FLAT_ENV != "0", "fdw" if _FLAT_ENV == "1" else _FLAT_ENV]  # on, modes ("f", "d", "w")


def _launch_geom(geom, mode: str = "f"):
    if not FLAT1X1[0] or mode not in FLAT1X1[1] or geom.R != 1 or geom.S != 1 or geom.stride != 1 or geom.pad != 0:
        return geom
    if geom.W & (geom.W - 1) == 0 and geom.W <= 128:
        return geom
    npix = geom.N * geom.H * geom.W
    if npix % 128:
        return geom
    return type(geom)(geom.G, 1, npix // 128, 128, geom.C, geom.K, 1, 1, 1, 0)


def _cfg(cfg: int) -> int:
    """Launch cfg with the engine bit: forced by a fixed engine; under "auto" the plan's own."""
    if _MATH[0] == "x6":
        return cfg | X6_BIT
    if _MATH[0] == "mfma32":
        return cfg & ~X6_BIT
    return cfg


_PLANS: dict = {}
_OVERRIDE: dict = {}
_MODE_NAMES = ("fwd", "dgrad", "wgrad")
# measured best plans per (mode, geometry) (scripts/conv_f32_tune.py on an MI355X)
_TUNED_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "f32_plans.json")
_TUNED: dict | None = None


def _tuned(mode: int, g):
    global _TUNED
    if _TUNED is None:
        _TUNED = {}
        if os.environ.get("DDL_F32_TUNED", "1") != "0" and os.path.exists(_TUNED_PATH):
            import json
            with open(_TUNED_PATH) as f:
                _TUNED = json.load(f).get("plans", {})
    key = f"{_MODE_NAMES[mode]}:{g.G},{g.N},{g.H},{g.W},{g.C},{g.K},{g.R},{g.S},{g.stride},{g.pad}"
    if _MATH[0] == "auto":
        p = _TUNED.get(f"auto:{key}")
        if p is not None:
            return cfg_of(p[0], p[1]) | (X6_BIT if p[3] == "x6" else 0), int(p[2])
        p = _TUNED.get(f"x6:{key}")
        return None if p is None else (cfg_of(p[0], p[1]) | X6_BIT, int(p[2]))
    if _MATH[0] != "mfma32":
        key = f"{_MATH[0]}:{key}"
    p = _TUNED.get(key)
    return None if p is None else (cfg_of(p[0], p[1]), int(p[2]))


# The vendor fp32 GEMM (torch.mm -> hipBLASLt) for plain-GEMM callers is an opt-in A/B only:
# DDL_F32_BLAS=1 (always) or "auto" (where a "blas:" entry of the plan table says so; the shipped
# table has none since round 6: every fp32 LLaMA linear product runs a native engine, see
# ops/llama_f32.py LINEAR). Default 0: never.
BLAS = [os.environ.get("DDL_F32_BLAS", "0")]


def vendor_gemm(mode: int, g) -> bool:
    if BLAS[0] in ("0", "1"):
        return BLAS[0] == "1"
    _tuned(mode, g)  # loads the table
    return f"blas:{_MODE_NAMES[mode]}:{g.G},{g.N},{g.H},{g.W},{g.C},{g.K},{g.R},{g.S},{g.stride},{g.pad}" in _TUNED


def set_plan(mode: int, geom, bp: int, bq: int, split: int, engine: str | None = None) -> None:
    """Pin a launch plan (tile BP x BQ, split-K slices[, engine under "auto": "x6", "mfma32", or
    "x6h" = the halo kernel, BQ 128]) for one (mode, geometry) — the tuner and the tests."""
    bits = {None: X6_BIT, "x6": X6_BIT, "x6h": X6_BIT | HALO_BIT, "mfma32": 0}[engine]
    _OVERRIDE[(mode, geom)] = (cfg_of(bp, bq) | bits, int(split))
    _PLANS.pop((mode, geom), None)


def clear_plan(mode: int, geom) -> None:
    _OVERRIDE.pop((mode, geom), None)
    _PLANS.pop((mode, geom), None)


# DDL_F32_RECORD=<path>: every (mode, geometry) a process plans is written there as JSON at exit,
# for scripts/conv_f32_tune.py --geoms-file (tune exactly the launches a workload makes)
_RECORD_PATH = os.environ.get("DDL_F32_RECORD", "")
_RECORDED: set = set()


def _write_record():
    import json
    rows = sorted({(m, (g.G, g.N, g.H, g.W, g.C, g.K, g.R, g.S, g.stride, g.pad)) for m, g in _RECORDED})
    with open(_RECORD_PATH, "w") as f:
        json.dump([{"mode": _MODE_NAMES[m], "geom": list(g)} for m, g in rows], f)


if _RECORD_PATH:
    import atexit
    atexit.register(_write_record)


def plan(mode: int, geom) -> tuple[int, int]:
    """(cfg, split) heuristic: 128-wide tiles where the dimension allows, then split-K until the
    grid has ~TARGET_WG workgroups (each slice keeping >= 8 reduction steps)."""
    key = (mode, geom)
    p = _PLANS.get(key)
    if p is not None:
        return p
    if _RECORD_PATH:
        _RECORDED.add(key)
    p = _OVERRIDE.get(key)
    if p is None and _HALO[0] and _MATH[0] != "mfma32" and halo_ok(mode, geom, auto=True):
        p = _halo_plan(mode, geom)
    if p is None:
        p = _tuned(mode, geom)
    if p is None:
        Pd, Qd, Kr, nph = _dims(mode, geom)
        bp = 128 if Pd > 64 else 64
        bq = 128 if Qd > 64 else 64
        tiles = -(-Pd // bp) * -(-Qd // bq) * nph * geom.G
        nk = -(-Kr // 16)
        split = 1
        while tiles * split < TARGET_WG and nk >= split * 2 * 8 and split < 64:
            split *= 2
        p = (cfg_of(bp, bq) | X6_BIT, split)
    _PLANS[key] = p
    return p


def _halo_plan(mode: int, geom) -> tuple[int, int]:
    """Halo kernel: a measured plan ('x6h:' entries of f32_plans.json, scripts/halo_plan_probe.py:
    e.g. BP 64 without split-K for the 16x16 layer at one client, 59 vs 78 us); otherwise BP 128
    where the output channels allow, 128-pixel tiles, split-K over the 16-channel chunks until
    ~TARGET_WG workgroups (each slice keeping >= 4 chunks)."""
    _tuned(mode, geom)  # loads the table
    if TARGET_WG != 1:  # TARGET_WG = 1 pins split-K off (the multi-rank rehearsal's plans)
        p = _TUNED.get(f"x6h:{_MODE_NAMES[mode]}:{geom.G},{geom.N},{geom.H},{geom.W},{geom.C},{geom.K},"
                       f"{geom.R},{geom.S},{geom.stride},{geom.pad}")
        if p is not None:
            return cfg_of(int(p[0]), int(p[1])) | X6_BIT | HALO_BIT, int(p[2])
    Pd, Qd, _, _ = _dims(mode, geom)
    SC = geom.C if mode == F_FWD else geom.K
    # BP 128 where the channels allow, except 4x4 images: their 8-image halo (43 KiB) with a BP 128
    # weight ring would leave one workgroup per CU
    bp = 128 if Pd > 64 and geom.Q > 4 else 64
    tiles = -(-Pd // bp) * -(-Qd // 128) * geom.G
    nch = SC // 16
    split = 1
    padded = geom.Q & (geom.Q - 1) != 0
    while not padded and tiles * split < TARGET_WG and nch >= split * 2 * 4 and split < 32:
        split *= 2
    return cfg_of(bp, 128) | X6_BIT | HALO_BIT, split


def _args(geom, **kw) -> _lib.ConvF32Args:
    a = _lib.ConvF32Args()
    a.gscale = 1.0
    for k, v in kw.items():
        setattr(a, k, v)
    a.G, a.N, a.H, a.W, a.C, a.K = geom.G, geom.N, geom.H, geom.W, geom.C, geom.K
    a.R, a.S, a.P, a.Q, a.stride, a.pad = geom.R, geom.S, geom.P, geom.Q, geom.stride, geom.pad
    return a


def _gs(t) -> int:
    return 0 if t is None else t.stride(0)


def _launch(a, mode: int, geom, device, split_k: int = 0, ws_role: str = "main") -> None:
    lib = _lib.kernels()
    cfg, split = plan(mode, geom)
    if split_k:
        split = split_k
    a.split_k = split
    cfg = _cfg(cfg)
    if cfg & HALO_BIT and not halo_ok(mode, geom):
        cfg &= ~HALO_BIT
    if split > 1:
        need = lib.ddl_convf32_workspace(ctypes.byref(a), mode, cfg)
        buf = workspace(device, ws_role)
        if need > buf.numel():
            a.split_k = split = 1  # plan-determined (same choice eager and captured)
        else:
            a.partial, a.partial_cap = buf.data_ptr(), buf.numel()
            if WG_FOLD[0] and not (cfg & HALO_BIT):  # the halo kernel keeps its epilogue launch
                t = _WS[f"{device}:{ws_role}:tickets"]
                a.tickets, a.tickets_cap = t.data_ptr(), t.numel()
    name = ("conv_fwd", "conv_dgrad", "conv_wgrad")[mode] + "_f32"
    if cfg & HALO_BIT:
        ws_buf = split_weights(a, mode, geom, device)
        a.wsplit, a.ws_gs = ws_buf.data_ptr(), ws_buf.stride(0)  # bytes
        check(lib.ddl_x6h(ctypes.byref(a), mode, cfg & ~HALO_BIT, stream()), name + "_halo")
        return
    check(lib.ddl_convf32(ctypes.byref(a), mode, cfg, stream()), name)


def split_weights(a, mode: int, geom, device) -> torch.Tensor:
    """The X6 operand image of the launch's weights (6 bytes per element: three bf16 planes per 16
    channels): FWD layout [G][K][R][S][C], DGRAD layout [G][C][R][S][K]. Inside an open
    :class:`PresplitScope` (a training step) the image the scope built at step start; otherwise
    rebuilt from the fp32 weights for this launch (the fused-SGD WGRAD updates them in place), into
    a stream-ordered temporary."""
    T = geom.R * geom.S
    layout = 0 if mode == F_FWD else 1
    scope = _PRESPLIT[0]
    if scope is not None:
        key = (int(a.w), layout, geom.G, geom.K, T, geom.C, int(a.w_gs))
        buf = scope.lookup(key)
        if buf is not None:
            return buf
    out = torch.empty(geom.G, geom.K * T * geom.C * 6, dtype=torch.uint8, device=device)
    check(_lib.kernels().ddl_x6_split_weights(a.w, out.data_ptr(), geom.G, geom.K, T, geom.C, 0 if mode == F_FWD else 1,
                                              a.w_gs, out.stride(0), 0, stream()), "x6_split_weights")
    return out


class _SplitDesc(ctypes.Structure):  # conv_x6h.hip SplitDesc
    _fields_ = [("w", ctypes.c_void_p), ("out", ctypes.c_void_p), ("w_gs", ctypes.c_longlong),
                ("o_gs", ctypes.c_longlong), ("G", ctypes.c_int), ("K", ctypes.c_int), ("T", ctypes.c_int),
                ("C", ctypes.c_int), ("layout", ctypes.c_int), ("blk0", ctypes.c_int), ("nblk", ctypes.c_int),
                ("pad_", ctypes.c_int)]


_PRESPLIT: list = [None]  # the open PresplitScope (one training step), or None
PRESPLIT = [os.environ.get("DDL_F32_PRESPLIT", "1") != "0"]
# Split the images the step's first layers need on the step's stream and the rest (later layers'
# FWD images, every DGRAD image) on a side stream, overlapped with those first layers; the step's
# stream joins the side stream at the first request of a deferred image. HEAD_FRAC: the share of
# the image volume split up front. OFF by default (DDL_F32_PRESPLIT_SIDE=1 enables it): measured
# 40.15k vs 40.29k samples/s at 8 clients, 23.99k vs 24.03k at 1 — the memory-bound split has no
# free CU slots beside the first layers' halo convs (registers / LDS full), so it only interleaves.
PRESPLIT_SIDE = [os.environ.get("DDL_F32_PRESPLIT_SIDE", "0") == "1"]
PRESPLIT_HEAD_FRAC = float(os.environ.get("DDL_F32_PRESPLIT_HEAD", "0.05"))
_SPLIT_STREAMS: dict = {}


class PresplitScope:
    """Every X6 weight image a training step needs, built by ONE launch at step start.

    The halo kernels read the weights as pre-split bf16 piece images (``split_weights``); per conv
    that was one small launch before each FWD and each DGRAD (23 per ResNet-18 step, ~5-14 us each
    at one client per GPU, on the critical path). A step's weights do not change between its
    forward and the DGRADs that read them (a direct-SGD WGRAD steps a layer's weights only after
    that layer's DGRAD), so all images can be made up front. The first step through a scope
    records the (weights, layout) pairs its halo launches ask for and splits them per launch as
    before; from then on the scope owns one persistent image per pair, refreshed by
    ``ddl_x6_split_weights_multi`` when the scope opens (a captured step replays that one launch).
    A request the recording did not see falls back to the per-launch split. Use it only around
    code whose weights stay fixed while it runs (``Net.train_step``), never around e.g. a GAN step
    that updates D between two forwards."""

    def __init__(self):
        self.keys: list = []
        self._seen: set = set()
        self.bufs: dict = {}
        self.tables: list = []  # [(device descriptor table, n descriptors, n blocks)]: head, tail
        self.tail: set = set()  # keys split on the side stream
        self._pending = None  # the side stream's event until the step's stream has waited on it
        self.state = "record"  # -> "ready" once the images and the descriptor tables exist
        self._prev = None

    def lookup(self, key):
        if self.state == "ready":
            if self._pending is not None and key in self.tail:
                torch.cuda.current_stream().wait_event(self._pending)
                self._pending = None
            return self.bufs.get(key)
        if key not in self._seen:
            self._seen.add(key)
            self.keys.append(key)
        return None

    def __enter__(self):
        self._prev = _PRESPLIT[0]
        if not PRESPLIT[0]:
            return self
        if self.state == "ready":
            lib = _lib.kernels()
            desc, n, nb = self.tables[0]
            check(lib.ddl_x6_split_weights_multi(ptr(desc), n, nb, stream()), "x6_split_weights_multi")
            if len(self.tables) > 1:
                cur = torch.cuda.current_stream()
                side = _SPLIT_STREAMS.get(cur.device)
                if side is None:
                    side = _SPLIT_STREAMS[cur.device] = torch.cuda.Stream(device=cur.device)
                side.wait_stream(cur)  # this step's weights (and the last step's image readers)
                desc, n, nb = self.tables[1]
                with torch.cuda.stream(side):
                    check(lib.ddl_x6_split_weights_multi(ptr(desc), n, nb, stream()), "x6_split_weights_multi")
                    ev = torch.cuda.Event()
                    ev.record(side)
                self._pending = ev
        _PRESPLIT[0] = self
        return self

    def __exit__(self, *exc):
        _PRESPLIT[0] = self._prev
        if self._pending is not None:  # join the side stream even if no deferred image was read
            torch.cuda.current_stream().wait_event(self._pending)
            self._pending = None
        if self.state == "record" and self.keys and not torch.cuda.is_current_stream_capturing() \
                and exc[0] is None:
            self._build()
        return False

    def _build(self):
        lib = _lib.kernels()
        if lib.ddl_x6_split_desc_size() != ctypes.sizeof(_SplitDesc):
            raise RuntimeError("ABI mismatch for SplitDesc")
        dev = torch.device("cuda", torch.cuda.current_device())
        vol = [k[2] * k[3] * k[4] * k[5] for k in self.keys]
        nhead = len(self.keys)
        if PRESPLIT_SIDE[0] and len(self.keys) > 1:  # first-requested keys up to HEAD_FRAC of the volume
            nhead, acc = 1, vol[0]
            while nhead < len(self.keys) and acc + vol[nhead] <= PRESPLIT_HEAD_FRAC * sum(vol):
                acc += vol[nhead]
                nhead += 1
        self.tail = set(self.keys[nhead:])
        self.tables = []
        for part in (self.keys[:nhead], self.keys[nhead:]):
            if not part:
                continue
            descs = (_SplitDesc * len(part))()
            blk = 0
            for i, key in enumerate(part):
                w, layout, G, K, T, C, w_gs = key
                buf = torch.empty(G, K * T * C * 6, dtype=torch.uint8, device=dev)
                self.bufs[key] = buf
                nblk = max(1, min(1024, -(-G * K * T * C // 16 // 256)))
                d = descs[i]
                d.w, d.out, d.w_gs, d.o_gs = w, buf.data_ptr(), w_gs, buf.stride(0)
                d.G, d.K, d.T, d.C, d.layout, d.blk0, d.nblk = G, K, T, C, layout, blk, nblk
                blk += nblk
            raw = torch.frombuffer(bytearray(bytes(descs)), dtype=torch.uint8)
            self.tables.append((raw.to(dev), len(part), blk))
        self.state = "ready"


def _store_identity(owner):
    """(data_ptr, numel, storage id) of the owner's weight store: the scope's image keys are raw
    weight pointers, valid only while the store they point into is the same allocation."""
    store = getattr(owner, "store", None)
    data = getattr(store, "data", None)
    if data is None:
        return None
    return data.data_ptr(), data.numel(), id(data.untyped_storage())


def presplit_scope(owner) -> "PresplitScope | contextlib.nullcontext":
    """The owner's (a Net's) PresplitScope for one training step (a no-op context off the fp32
    device path or with DDL_F32_PRESPLIT=0). A scope is rebuilt (re-recorded) whenever the owner's
    weight store was re-materialised since it recorded: its persistent images and descriptor table
    are keyed on the old weight pointers, which a reallocation would turn into reads of freed
    memory (or, worse, of a new tensor the allocator placed at the same address)."""
    sig = _store_identity(owner)
    sc = getattr(owner, "_f32_presplit", None)
    if sc is None or getattr(owner, "_f32_presplit_sig", None) != sig:
        sc = PresplitScope()
        owner._f32_presplit = sc
        owner._f32_presplit_sig = sig
    return sc


def _slots(a, mode: int, geom) -> int:
    cfg, _ = plan(mode, geom)
    if uses_halo(mode, geom):  # the halo kernel's own tiles (row-padded widths included)
        return int(_lib.kernels().ddl_x6h_slots(ctypes.byref(a), mode))
    return int(_lib.kernels().ddl_convf32_slots(ctypes.byref(a), mode, _cfg(cfg)))


def slot_rows(mode: int, geom) -> int:
    """Output pixels per statistics slot of a launch: the tile's BQ, or on the halo kernel with a
    row-padded width its real pixels, (128 / padded width) rows of W."""
    cfg, _ = plan(mode, geom)
    bq = ((_cfg(cfg) >> 8) & 0xFF) * 16
    if uses_halo(mode, geom) and geom.Q & (geom.Q - 1):
        return bq // (1 << (geom.Q - 1).bit_length()) * geom.Q
    return bq


def _xform(in_bn):
    if in_bn is None:
        return {}
    sc, sh = in_bn
    assert sc.is_contiguous() and sh.is_contiguous()
    return dict(in_scale=ptr(sc), in_shift=ptr(sh), in_relu=1)


def conv_fwd(x, w, geom, bias=None, relu=False, stats=None, out=None, residual=None, in_bn=None, split_k=0):
    y = out if out is not None else torch.empty(geom.G, geom.N, geom.P, geom.Q, geom.K, dtype=torch.float32,
                                                device=x.device)
    if residual is not None and (residual.stride(0) != y.stride(0) or not residual.is_contiguous()):
        residual = residual.contiguous()
    geom = _launch_geom(geom, "f")
    a = _args(geom, x=ptr(x), w=ptr(w), out=ptr(y), bias=ptr(bias), residual=ptr(residual),
              x_gs=_gs(x), w_gs=_gs(w), out_gs=_gs(y), bias_gs=_gs(bias), relu=int(bool(relu)), **_xform(in_bn))
    if stats is not None:
        st = torch.empty(geom.G, _slots(a, F_FWD, geom), 2, geom.K, dtype=torch.float32, device=x.device)
        a.stats = ptr(st)
        if isinstance(stats, SlotStats):
            stats.t = st
            stats.rows = slot_rows(F_FWD, geom)
        else:
            raise TypeError("fp32 conv statistics go to a SlotStats (Fn.stats_buffer(..., like=x))")
    _launch(a, F_FWD, geom, x.device, split_k)
    return y


def conv_dgrad(dy, w, geom, residual=None, mask=None, out=None, bn=None, mask_bn=None, residual_sub=1,
               split_k=0, dy_bn=None, dy_bn_out=None):
    """dy_bn = (x_bn, coef): the dY operand is the following BN's backward A * dy + B * x_bn + C
    (bn_backward_coef), applied inside the halo kernel as dY is staged (written to ``dy_bn_out``
    too, for the layer's WGRAD); launches off the halo kernel materialise it first."""
    dx = out if out is not None else torch.empty(geom.G, geom.N, geom.H, geom.W, geom.C, dtype=torch.float32,
                                                 device=dy.device)
    if residual_sub == 1:
        geom = _launch_geom(geom, "d")
    kw = {}
    if dy_bn is not None:
        xb, coef = dy_bn
        assert xb.is_contiguous() and coef.is_contiguous() and xb.shape == dy.shape and dy.is_contiguous()
        if uses_halo(F_DGRAD, geom) and split_k == 0:
            kw.update(dyb_x=ptr(xb), dyb_coef=ptr(coef), dyb_out=ptr(dy_bn_out))
        else:
            dy = coef_apply(dy, xb, coef, out=dy_bn_out)
    if residual is not None and residual_sub == 2 and geom.H & 1 and uses_halo(F_DGRAD, geom) \
            and (split_k or plan(F_DGRAD, geom)[1]) <= 1:
        # the halo epilogue reads the compact grid on even-height images only (conv_x6h.hip fepi_t)
        full = torch.zeros_like(dx)
        full[:, :, ::2, ::2] = residual
        residual, residual_sub = full, 1
    if residual is not None:
        if residual_sub == 2:
            want = (geom.G, geom.N, (geom.H + 1) // 2, (geom.W + 1) // 2, geom.C)
            assert tuple(residual.shape) == want, (tuple(residual.shape), want)
            residual = residual.contiguous()
            kw.update(res_sub=2, res_gs=residual.stride(0))
        elif residual.stride(0) != dx.stride(0) or not residual.is_contiguous():
            residual = residual.contiguous()
    if mask is not None and (mask.stride(0) != dx.stride(0) or not mask.is_contiguous()):
        mask = mask.contiguous()
    if bn is not None:
        x, mean, rstd = bn
        assert x.is_contiguous() and x.stride(0) == dx.stride(0) and mean.is_contiguous() and rstd.is_contiguous()
        kw.update(bn_x=ptr(x), bn_mean=ptr(mean), bn_rstd=ptr(rstd))
        if mask_bn is not None:
            sc, sh = mask_bn
            assert sc.is_contiguous() and sh.is_contiguous() and sc.numel() == geom.G * geom.C
            kw.update(mask_scale=ptr(sc), mask_shift=ptr(sh))
    a = _args(geom, w=ptr(w), dy=ptr(dy), out=ptr(dx), residual=ptr(residual), mask=ptr(mask),
              w_gs=_gs(w), dy_gs=_gs(dy), out_gs=_gs(dx), **kw)
    part = None
    if bn is not None:
        part = torch.empty(geom.G, _slots(a, F_DGRAD, geom), 2, geom.C, dtype=torch.float32, device=dy.device)
        a.stats = ptr(part)
    _launch(a, F_DGRAD, geom, dy.device, split_k)
    return dx if bn is None else (dx, part)


# conv_x6hw.hip: the halo-staged X6 WGRAD (stride-1 "same" convs, K % 64, C % 32, OW a power of
# two >= 8). It beats conv_f32.hip on images >= 16 wide (8 clients, c64 / c128: 0.49 / 0.46 ms vs
# 0.65 / 0.50 ms) and loses on 8x8 (c256: 0.55 vs 0.50 ms: the halo is 60 % padding there),
# profiles/x6hw_wgrad_r4.txt. DDL_F32_HALO_WGRAD=0 disables it; HW_MIN_W is the width rule.
HALO_WGRAD = [os.environ.get("DDL_F32_HALO_WGRAD", "1") != "0"]
HW_MIN_W = int(os.environ.get("DDL_F32_HW_MIN_W", "16"))
HW_TARGET_WG = int(os.environ.get("DDL_F32_HW_TARGET_WG", "256"))  # one workgroup per CU (LDS-bound)


def uses_halo_wgrad(geom) -> bool:
    """Does conv_wgrad take the halo WGRAD (conv_x6hw.hip) for this geometry?"""
    a = _args(geom)
    return HALO_WGRAD[0] and _MATH[0] != "mfma32" and geom.W >= HW_MIN_W \
        and bool(_lib.kernels().ddl_x6hw_ok(ctypes.byref(a)))


def _halo_wgrad(a, geom, device, split_k: int, ws_role: str) -> bool:
    """Launch the halo WGRAD when it takes this geometry: a measured slice count ('x6hw:' entries of
    f32_plans.json, scripts/halo_plan_probe.py), else split-K over pixel tiles until ~one
    workgroup per CU (each slice keeping >= 3 tiles); slices folded in slice order."""
    if not (HALO_WGRAD[0] and _MATH[0] != "mfma32") or geom.W < HW_MIN_W \
            or not _lib.kernels().ddl_x6hw_ok(ctypes.byref(a)):
        return False
    lib = _lib.kernels()
    ntile = int(lib.ddl_x6hw_tiles(ctypes.byref(a)))
    base = (geom.K // 64) * (geom.C // 32) * geom.G
    split = split_k or 1
    if not split_k and TARGET_WG != 1:
        _tuned(F_WGRAD, geom)  # loads the table
        p = _TUNED.get(f"x6hw:wgrad:{geom.G},{geom.N},{geom.H},{geom.W},{geom.C},{geom.K},{geom.R},{geom.S},"
                       f"{geom.stride},{geom.pad}")
        if p is not None:
            split_k = split = int(p[0])
    if not split_k:
        target = min(HW_TARGET_WG, TARGET_WG)  # TARGET_WG = 1 pins split-K off for every conv
        while base * split < target and ntile >= split * 2 * 3 and split < 128:
            split *= 2
    n = geom.K * geom.R * geom.S * geom.C
    if split > 1:
        buf = workspace(device, ws_role)
        while split > 1 and split * geom.G * n > buf.numel():
            split //= 2  # the largest split the workspace holds (plan-determined: eager == captured)
        if split > 1:
            a.partial, a.partial_cap = buf.data_ptr(), buf.numel()
    a.split_k = split
    check(lib.ddl_x6hw(ctypes.byref(a), stream()), "conv_wgrad_f32_halo")
    if split > 1:
        check(lib.ddl_convf32_wgrad_reduce(a.partial, a.out, a.out_gs, geom.G, n, split, a.accumulate, a.gscale,
                                           stream()), "conv_wgrad_f32_halo_reduce")
    return True


def conv_wgrad(dy, x, geom, dw, accumulate=True, gscale=1.0, in_bn=None, split_k=0, ws_role="main"):
    if not accumulate and gscale != 1.0:
        raise ValueError("a scaled WGRAD must accumulate (it adds into the master weights)")
    geom = _launch_geom(geom, "w")
    a = _args(geom, x=ptr(x), dy=ptr(dy), out=ptr(dw), x_gs=_gs(x), dy_gs=_gs(dy), out_gs=_gs(dw),
              accumulate=int(bool(accumulate)), gscale=float(gscale), **_xform(in_bn))
    if (F_WGRAD, geom) not in _OVERRIDE and _halo_wgrad(a, geom, dy.device, split_k, ws_role):
        return dw
    _launch(a, F_WGRAD, geom, dy.device, split_k, ws_role)
    return dw


# --------------------------------------------------------------------------------------- BN
def _bnf_args(stats, gamma, beta, running_mean, running_var, count, eps, momentum, training, outs, G, C,
              tile_rows=0):
    a = _lib.BNFArgs()
    a.tile_rows = int(tile_rows)
    a.stats, a.gamma, a.beta = ptr(stats), ptr(gamma), ptr(beta)
    a.running_mean, a.running_var = ptr(running_mean), ptr(running_var)
    a.scale, a.shift, a.mean, a.rstd = (ptr(outs[i]) for i in range(4))
    a.gs_param = _gs(gamma) if gamma is not None else _gs(beta)
    a.gs_buf = _gs(running_mean)
    a.G, a.C, a.count = G, C, int(count)
    a.eps, a.momentum, a.training = float(eps), float(momentum), int(training)
    a.stripes = stats.shape[1] if stats is not None else 0
    return a


def bn_finalize_many(items, eps=1e-5, momentum=0.1, training=True):
    """items: [(stats SlotStats | tensor | None, gamma, beta, running_mean, running_var, count, G, C), ...]
    (one or two BatchNorms, one launch) -> [(scale, shift, mean, rstd), ...]."""
    dev = items[0][1].device if items[0][1] is not None else items[0][3].device
    args, outs = [], []
    for stats, gamma, beta, rm, rv, count, G, C in items:
        t = stats.t if isinstance(stats, SlotStats) else stats
        rows = stats.rows if isinstance(stats, SlotStats) else 0
        if training:
            assert t is not None and t.is_contiguous(), "fp32 BN statistics missing (conv not run?)"
        o = torch.empty(4, G, C, dtype=torch.float32, device=dev)
        args.append(_bnf_args(t if training else None, gamma, beta, rm, rv, count, eps, momentum, training, o, G, C,
                              rows))
        outs.append(o)
    b = ctypes.byref(args[1]) if len(args) > 1 else None
    check(_lib.kernels().ddl_bnf_finalize(ctypes.byref(args[0]), b, stream()), "bn_finalize_f32")
    return [(o[0], o[1], o[2], o[3]) for o in outs]


def bn_apply(x, scale, shift, r=None, rscale=None, rshift=None, act=0, out=None):
    assert x.is_contiguous() and (r is None or r.is_contiguous())
    y = out if out is not None else torch.empty_like(x)
    G, C = x.shape[0], x.shape[-1]
    check(_lib.kernels().ddl_bnf_apply(ptr(x), ptr(scale), ptr(shift), ptr(r), ptr(rscale), ptr(rshift), ptr(y),
                                       x[0].numel(), C, G, act, stream()), "bn_apply_f32")
    return y


def reduce_slots(M: int, C: int, G: int) -> int:
    return int(_lib.kernels().ddl_bnf_reduce_slots(int(M), int(C), int(G)))


def bn_bwd_reduce_part(dy, ymask, x, mean, rstd):
    G, C = x.shape[0], x.shape[-1]
    M = x[0].numel() // C
    part = torch.empty(G, reduce_slots(M, C, G), 2, C, dtype=torch.float32, device=x.device)
    check(_lib.kernels().ddl_bnf_reduce(ptr(dy), ptr(ymask), ptr(x), ptr(mean), ptr(rstd), ptr(part), M, C, G,
                                        stream()), "bn_bwd_reduce_f32")
    return part


def bn_stats(x):
    G, C = x.shape[0], x.shape[-1]
    M = x[0].numel() // C
    st = SlotStats()
    st.t = torch.empty(G, reduce_slots(M, C, G), 2, C, dtype=torch.float32, device=x.device)
    check(_lib.kernels().ddl_bnf_stats(ptr(x), ptr(st.t), M, C, G, stream()), "bn_stats_f32")
    return st


def _bwd_args(x, mean, rstd, gamma, dgamma, dbeta, part, dx, fold_slots: int = 0, coef=None):
    """fold_slots: size the two-level fold's workspace for this many slots (0: part's own).
    coef: where the folded (A | B | C) coefficients go (default: launch-local scratch)."""
    G, C = x.shape[0], x.shape[-1]
    t = _lib.BNFBwdArgs()
    if coef is None:
        coef = ws.scratch_uninit((G, 3, C), x.device)  # the fold writes every coefficient
    gs = _gs(gamma) if gamma is not None else 0
    if dgamma is not None or dbeta is not None:
        gd = _gs(dgamma) if dgamma is not None else _gs(dbeta)
        assert gamma is None or gd == gs, "gamma and its gradient must share the group stride"
        gs = gd
    t.x, t.mean, t.rstd, t.gamma = ptr(x), ptr(mean), ptr(rstd), ptr(gamma)
    t.dgamma, t.dbeta, t.part, t.coef, t.dx, t.gs_param = ptr(dgamma), ptr(dbeta), ptr(part), ptr(coef), ptr(dx), gs
    t.slots = part.shape[1] if part is not None else 0
    S = max(fold_slots, t.slots)
    fws = None
    if FOLD2[0] and S > 0:
        fws = torch.empty(int(_lib.kernels().ddl_bnf_fold_ws(S, C, G)), dtype=torch.float64, device=x.device)
        t.fold_ws = fws.data_ptr()
        if FOLD1L[0] and x.is_cuda:
            t.tickets = _fold_tickets(x.device, int(_lib.kernels().ddl_bnf_fold_tickets(C, G)))
    t._keep = (coef, fws)  # scratch that must outlive the launch (its memory would be reused otherwise)
    return t


# BN-backward coefficient fold: two small-block levels (DDL_F32_FOLD2=0: the one-level fold), in
# ONE launch whose last-arriving block folds the level-1 partials (DDL_F32_FOLD1L=0: two launches)
FOLD2 = [os.environ.get("DDL_F32_FOLD2", "1") != "0"]
FOLD1L = [os.environ.get("DDL_F32_FOLD1L", "1") != "0"]
_TICKETS: dict = {}


TICKETS_N = 1 << 16  # >= 2 * G * C / 32 of any BN (G = 64 clients at C = 512: 2048)


def _dev_key(device) -> str:
    d = torch.device(device)
    return f"cuda:{d.index if d.index is not None else torch.cuda.current_device()}"


def _fold_tickets(device, n: int) -> int:
    """Zeroed arrival counters of the one-launch fold, one buffer per device: every fold returns
    its counters to zero, so the BN backwards share them — which requires every fold of a device
    to run on ONE stream (they do: the step's main stream, eager or captured; the side stream only
    carries conv WGRADs). ``fold_tickets_clean`` checks the invariant after a step (tests).
    Allocated eagerly with the split-K workspace (a first use inside a graph capture raises)."""
    key = _dev_key(device)
    buf = _TICKETS.get(key)
    if buf is None:
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("fp32 BN fold counters first requested inside a graph capture: run one eager "
                               "step (or functional_f32.ensure_workspace) before capturing")
        buf = torch.zeros(TICKETS_N, dtype=torch.int32, device=device)
        _TICKETS[key] = buf
    if n > buf.numel():
        raise ValueError(f"BN fold needs {n} counters (> {buf.numel()})")
    return buf.data_ptr()


def fold_tickets_clean() -> bool:
    """Debug check: every BN-fold arrival counter is back to zero (a fold that was aborted, or two
    folds racing on one counter set, would leave counts behind and corrupt later coefficients)."""
    torch.cuda.synchronize()
    return all(int(b.abs().sum().item()) == 0 for b in _TICKETS.values())


def bn_backward(dy, ymask, x, mean, rstd, gamma, dgamma=None, dbeta=None, emit_dym=False, part=None):
    G, C = x.shape[0], x.shape[-1]
    M = x[0].numel() // C
    assert dy.is_contiguous() and x.is_contiguous()
    do_reduce = part is None
    if do_reduce:
        part = torch.empty(G, reduce_slots(M, C, G), 2, C, dtype=torch.float32, device=x.device)
    dx = torch.empty_like(x)
    dym = torch.empty_like(x) if emit_dym else None
    a = _bwd_args(x, mean, rstd, gamma, dgamma, dbeta, part, dx)
    check(_lib.kernels().ddl_bnf_backward(ptr(dy), ptr(ymask), ctypes.byref(a), None, ptr(dym), M, C, G,
                                          int(do_reduce), stream()), "bn_backward_f32")
    return (dx, dym) if emit_dym else dx


# BN backward folded into the consuming DGRAD (DDL_F32_BNFOLD=0: separate apply pass)
BNFOLD = [os.environ.get("DDL_F32_BNFOLD", "1") != "0"]


def bn_backward_coef(dy, x, mean, rstd, gamma, dgamma=None, dbeta=None, part=None):
    """The BN backward WITHOUT its apply pass: d(gamma), d(beta) accumulated and the per-channel
    coefficients coef [G, 3, C] = (A | B | C) of dx = A * dy + B * x + C returned, for a consumer
    that applies them on the fly (conv_dgrad(dy_bn=(x, coef)))."""
    G, C = x.shape[0], x.shape[-1]
    M = x[0].numel() // C
    assert dy.is_contiguous() and x.is_contiguous()
    do_reduce = part is None
    if do_reduce:
        part = torch.empty(G, reduce_slots(M, C, G), 2, C, dtype=torch.float32, device=x.device)
    coef = torch.empty(G, 3, C, dtype=torch.float32, device=x.device)
    a = _bwd_args(x, mean, rstd, gamma, dgamma, dbeta, part, None, coef=coef)
    check(_lib.kernels().ddl_bnf_backward(ptr(dy), None, ctypes.byref(a), None, None, M, C, G, int(do_reduce),
                                          stream()), "bn_backward_coef_f32")
    return coef


def coef_apply(dy, x, coef, out=None):
    """out = A * dy + B * x + C (coef from bn_backward_coef): the apply pass, for consumers that
    cannot fuse it."""
    G, C = x.shape[0], x.shape[-1]
    out = out if out is not None else torch.empty_like(x)
    check(_lib.kernels().ddl_bnf_coef_apply(ptr(dy), ptr(x), ptr(coef), ptr(out), x[0].numel() // C, C, G, stream()),
          "bnf_coef_apply")
    return out


def uses_halo(mode: int, geom) -> bool:
    cfg, _ = plan(mode, geom)
    return bool(_cfg(cfg) & HALO_BIT) and halo_ok(mode, geom)


def bn_backward2(dy, bn_a, bn_b):
    """bn_* = (x, mean, rstd, gamma, dgamma, dbeta, part) -> (dx_a, dx_b); dy already masked."""
    xa = bn_a[0]
    G, C = xa.shape[0], xa.shape[-1]
    M = xa[0].numel() // C
    assert bn_b[0].shape == xa.shape and dy.is_contiguous()
    outs, args = [], []
    smax = max(bn_a[6].shape[1], bn_b[6].shape[1])
    for x, mean, rstd, gamma, dgamma, dbeta, part in (bn_a, bn_b):
        dx = torch.empty_like(x)
        args.append(_bwd_args(x, mean, rstd, gamma, dgamma, dbeta, part, dx, fold_slots=smax))
        outs.append(dx)
    check(_lib.kernels().ddl_bnf_backward(ptr(dy), None, ctypes.byref(args[0]), ctypes.byref(args[1]), None, M, C,
                                          G, 0, stream()), "bn_backward2_f32")
    return outs[0], outs[1]


def avgpool_bwd_bn(dy, x, bn):
    c, mean, rstd = bn
    G, N, H, W, C = x.shape
    assert x.is_contiguous() and c.is_contiguous() and dy.is_contiguous()
    dx = torch.empty_like(x)
    part = torch.empty(G, reduce_slots(N * H * W, C, G), 2, C, dtype=torch.float32, device=x.device)
    check(_lib.kernels().ddl_avgpoolf_bwd_bn(ptr(dy), ptr(x), ptr(c), ptr(mean), ptr(rstd), ptr(dx), ptr(part),
                                             G, N, H * W, C, stream()), "avgpool_bwd_bn_f32")
    return dx, part


def channel_sum(x, out):
    """out[G, C] (view, fp32) += per-channel sum of x [G, ..., C]: slots + fixed-order fold."""
    G, C = x.shape[0], x.shape[-1]
    M = x[0].numel() // C
    assert x.is_contiguous()
    part = torch.empty(G, reduce_slots(M, C, G), 2, C, dtype=torch.float32, device=x.device)
    check(_lib.kernels().ddl_bnf_channel_sum(ptr(x), ptr(out), _gs(out), ptr(part), M, C, G, stream()),
          "channel_sum_f32")
    return out


def head_train_ok(C: int, ncls: int) -> bool:
    return C % 4 == 0 and C // 4 <= 256 and 256 % (C // 4) == 0 and 1 <= ncls <= 64 and \
        (2 * C + 64 + 2048 + ncls * C) * 4 <= 64 * 1024


def head_train(x, w, b, labels, ncls: int, scale: float, dw, db, bn=None, with_correct=False):
    G, N, H, W, C = x.shape
    dev = x.device
    assert x.is_contiguous() and labels.is_contiguous() and head_train_ok(C, ncls)
    loss = torch.empty(G, dtype=torch.float32, device=dev)
    correct = torch.empty(G, dtype=torch.int32, device=dev) if with_correct else None
    dx = torch.empty_like(x)
    a = _lib.HeadFArgs()
    a.x, a.w, a.b, a.labels = ptr(x), ptr(w), ptr(b), ptr(labels)
    a.loss, a.correct, a.dw, a.db, a.dx = ptr(loss), ptr(correct), ptr(dw), ptr(db), ptr(dx)
    a.w_gs, a.dw_gs = _gs(w), _gs(dw)
    a.b_gs, a.db_gs = (_gs(b), _gs(db)) if b is not None else (0, 0)
    part = None
    if bn is not None:
        c, mean, rstd = bn
        assert c.is_contiguous() and mean.is_contiguous() and rstd.is_contiguous()
        part = torch.empty(G, N, 2, C, dtype=torch.float32, device=dev)
        a.c, a.mean, a.rstd, a.part = ptr(c), ptr(mean), ptr(rstd), ptr(part)
    pooled = torch.empty(G, N, C, dtype=torch.float32, device=dev)
    dlog = torch.empty(G, N, 64, dtype=torch.float32, device=dev)
    rl = torch.empty(G, N, dtype=torch.float32, device=dev)
    rh = torch.empty(G, N, dtype=torch.int32, device=dev)
    a.pooled, a.dlog, a.row_loss, a.row_hit = ptr(pooled), ptr(dlog), ptr(rl), ptr(rh)
    a.G, a.N, a.HW, a.C, a.ncls, a.scale = G, N, H * W, C, ncls, float(scale)
    check(_lib.kernels().ddl_headf_train(ctypes.byref(a), stream()), "head_train_f32")
    return loss, correct, dx, part


def conv_flops(geom) -> int:
    return 2 * geom.G * geom.N * geom.P * geom.Q * geom.K * geom.R * geom.S * geom.C


__all__ = [n for n in dir() if not n.startswith("_") and n not in ("ctypes", "math", "os", "torch")]
