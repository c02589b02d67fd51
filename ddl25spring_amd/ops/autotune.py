"""Per-shape conv tile autotuner (on-device, first eager use).

The conv kernels have a built-in heuristic (conv_igemm.hip: tile by channel count, small-grid
fallbacks, automatic halo / split-K), but the best tile moves with the client count per GPU: at
1-8 clients per GPU the same ResNet-18 layer has a different winner (profiles/conv_halo_sweep_*,
conv_wgrad_halo_r1.log; the FedAvg scaling runs put 8, 4, 2 and 1 clients on a GPU). So the first
EAGER call of each (mode, shape, fused-epilogue) key times the heuristic and a short list of
candidate tiles (streamed, halo-staged, halo WGRAD split counts) on scratch outputs, a few
launches captured in a HIP graph and replayed (GPU time, not host launch cost), and caches the
fastest. Later calls — including the ones
captured into the training step's HIP graph — use the cached pick. A key first met during graph
capture runs the heuristic (nothing is timed inside a capture).

DDL_CONV_AUTOTUNE=0 disables it (the heuristic everywhere).
"""
from __future__ import annotations

import os

import torch

from . import workspace as ws
from ..runtime.graphs import CAPTURE_MODE

ENABLED = os.environ.get("DDL_CONV_AUTOTUNE", "1") != "0"
LOG = os.environ.get("DDL_TUNE_LOG", "0") == "1"  # print every candidate's time (stderr)
EAGER_TIMING = os.environ.get("DDL_TUNE_EAGER", "0") == "1"
_CACHE: dict = {}

_FD_TILES = [(64, 128, 32, 4), (128, 128, 32, 3), (128, 128, 64, 2), (128, 256, 32, 2),
             (48, 256, 64, 2), (64, 128, 64, 3), (64, 64, 64, 3), (128, 64, 64, 3), (48, 256, 32, 4),
             (256, 128, 32, 3)]
_FD_HALO = [(48, 256, 4), (48, 128, 4), (128, 128, 4)]
WIDE_SPLIT = os.environ.get("DDL_TUNE_WIDE_SPLIT", "1") != "0"
# WGRAD re-fetches dy once per column tile and x once per (row tile, tap): the 256-wide tiles
# halve one of the two on the deep layers (512 x 4608 outputs)
_WG_TILES = [(128, 128, 32, 3), (64, 128, 32, 4), (64, 64, 64, 3), (128, 64, 64, 3), (128, 128, 64, 2),
             (256, 128, 32, 3), (128, 256, 32, 3), (256, 128, 32, 2), (128, 256, 32, 2)]


def _cfg(bp, bq, bk, ns, halo=False):
    from .functional import conv_cfg
    return conv_cfg(bp, bq, bk, ns, halo)


def candidates(mode: str, geom, accumulate: bool = True) -> list:
    """(cfg, splits) pairs; cfg None = the kernel heuristic."""
    from .functional import halo_eligible
    out = [(None, 0)]
    if mode in ("fwd", "dgrad"):
        red = geom.C if mode == "fwd" else geom.K
        out += [(_cfg(*t), 0) for t in _FD_TILES if red % t[2] == 0]
        out += [(_cfg(bp, bq, 32, ns, True), 0) for bp, bq, ns in _FD_HALO
                if halo_eligible(geom, bq, ns) and red % 32 == 0]
        if geom.R * geom.S * red >= 2304:  # deep reductions: split-K (+ its epilogue pass) too
            out += [(None, s) for s in (2, 4, 8)]
            if red % 64 == 0:
                out += [(_cfg(64, 64, 64, 3), s) for s in (2, 4)]
                # wide tiles at split-K depths: on one client's 4x4 / 8x8 layers the 64x64 tiles
                # re-read every weight slab once per 64-pixel column through L2 (layer 4: 236 MB
                # per conv); 128-wide tiles halve that, split-K restores the workgroup count
                if WIDE_SPLIT and geom.G * geom.N * geom.P * geom.Q <= 6400:
                    out += [(_cfg(*t), s) for t in ((128, 128, 64, 2), (128, 64, 64, 3), (64, 128, 64, 3))
                            for s in (2, 4, 8)]
    else:
        out += [(_cfg(*t), 0) for t in _WG_TILES if accumulate]
        if accumulate:  # the heuristic tile at explicit split-K depths (small grids: 1-2 clients)
            nk = geom.N * geom.P * geom.Q // 32
            out += [(None, s) for s in (4, 8, 16, 32, 64) if s <= max(1, nk // 8)]
            # and the small tiles at explicit depths (few tiles per client: deep layers, 1 client)
            out += [(_cfg(*t), s) for t in ((64, 64, 64, 3), (128, 64, 64, 3), (64, 128, 32, 4))
                    for s in (8, 16, 32) if s <= max(1, nk // 8)]
        if accumulate and wgrad_halo_eligible(geom):
            tiles = (geom.K // 64) * (geom.C // 32) * geom.G
            nk = geom.N * geom.H * geom.W // 32
            sp = max(1, -(-512 // tiles))
            for s in sorted({max(1, sp // 2), sp, 2 * sp, 4 * sp}):
                if s <= max(1, nk // 8):
                    out.append((_cfg(64, 288, 32, 4, True), s))  # 5-6 stages: no faster
    return out


def wgrad_halo_eligible(g) -> bool:
    """Mirror of conv_igemm.hip ``wgrad_halo_ok``."""
    return ((g.stride, g.R, g.S, g.pad) == (1, 3, 3, 1) and g.W in (8, 16, 32)
            and g.H % (32 // g.W) == 0 and g.K % 64 == 0 and g.C % 32 == 0)


def _key(mode, geom, flags):
    return (mode, geom.G, geom.N, geom.H, geom.W, geom.C, geom.K, geom.R, geom.S, geom.stride,
            geom.pad, flags)


def _time(run, cfg, sp, reps=8) -> float:
    """GPU time per launch: ``reps`` launches captured in one HIP graph and replayed. Timing eager
    launches measured the host instead on few-client shapes, whose kernels (5-25 us) are shorter
    than the Python + launch cost of a call: the picks then varied run to run (a 1-client layer-1
    forward drew a 128x256 tile at 25 us in one run, 64x256 at 19.5 us in another)."""
    run(cfg, sp)  # warm (and validity: raises on an ineligible tile), outside the capture
    if EAGER_TIMING:  # the round-1 method, kept for A/B
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(4):
            run(cfg, sp)
        b.record()
        b.synchronize()
        return a.elapsed_time(b) / 4
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, capture_error_mode=CAPTURE_MODE):
        for _ in range(reps):
            run(cfg, sp)
    graph.replay()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(3):
        graph.replay()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / (3 * reps)


def pick(mode: str, geom, flags: tuple, run, accumulate: bool = True):
    """The cached (cfg, splits) for this key, tuning it now if allowed. ``run(cfg, splits)`` must
    launch the op with scratch outputs (cfg None = heuristic)."""
    key = _key(mode, geom, flags)
    hit = _CACHE.get(key)
    if hit is not None:
        return hit
    if not ENABLED or torch.cuda.is_current_stream_capturing():
        return (None, 0)
    from ._lib import KernelError
    saved = ws._CURRENT
    ws._CURRENT = None  # scratch sums from torch.zeros, not the step arena
    try:
        best, best_t = (None, 0), float("inf")
        for cfg, sp in candidates(mode, geom, accumulate):
            try:
                t = _time(run, cfg, sp)
            except KernelError:
                continue
            if LOG:
                import sys
                print(f"[tune] {key} cfg={cfg} splits={sp} {t * 1e3:.1f} us", file=sys.stderr)
            if t < best_t * 0.97 or (cfg is None and t < best_t):  # ties keep the heuristic
                best, best_t = (cfg, sp), t
    finally:
        ws._CURRENT = saved
    _CACHE[key] = best
    return best


def pick_pair(tag, geom, dpick, wpick, supported, run_pair, run_seq, dmenu, wmenu):
    """Paired launch of two independent convs (functional.conv_dgrad_wgrad: DGRAD + WGRAD;
    functional.conv_fwd2: FWD + FWD): the fastest of the two tuned single launches back to back
    (-> None) and the paired kernels over (op A's tuned pick or a menu tile) x (op B's tuned pick or
    a menu tile) -> (cfg_a, split_a, cfg_b, split_b)."""
    key = _key("pair", geom, tag)
    if key in _CACHE:
        return _CACHE[key]
    if not ENABLED or torch.cuda.is_current_stream_capturing():
        return None
    from ._lib import KernelError
    saved = ws._CURRENT
    ws._CURRENT = None
    try:
        best, best_t = None, _time(lambda c, s: run_seq(), None, 0)
        seen = set()
        for dc, dsp in [dpick] + list(dmenu):
            for wc, wsp in [wpick] + list(wmenu):
                cand = (dc, dsp, wc, wsp)
                if cand in seen or not supported(*cand):
                    continue
                seen.add(cand)
                try:
                    t = _time(lambda c, s: run_pair(cand), None, 0)
                except KernelError:
                    continue
                if t < best_t * 0.97:
                    best, best_t = cand, t
    finally:
        ws._CURRENT = saved
    _CACHE[key] = best
    return best


def cache() -> dict:
    return dict(_CACHE)
