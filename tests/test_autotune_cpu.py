"""Conv autotuner bookkeeping (no GPU): candidate lists respect each kernel family's contract,
the heuristic is always a candidate, and picks are cached per (mode, shape, epilogue) key."""
from ddl25spring_amd.ops import autotune
from ddl25spring_amd.ops import functional as Fn
from ddl25spring_amd.ops.functional import ConvGeom


def _decode(cfg):
    ns = (cfg >> 24) & 0xFF
    return (cfg & 0xFF) * 16, ((cfg >> 8) & 0xFF) * 16, (cfg >> 16) & 0xFF, ns & 0x3F, bool(ns & 0x40)


def test_candidates_respect_kernel_contracts():
    g = ConvGeom(G=8, N=100, H=32, W=32, C=64, K=64, R=3, S=3, stride=1, pad=1)
    for mode in ("fwd", "dgrad", "wgrad"):
        cands = autotune.candidates(mode, g)
        assert cands[0] == (None, 0)
        halos = [c for c, _ in cands[1:] if c is not None and _decode(c)[4]]
        assert halos, mode  # layer-1 shape admits halo tiles in every mode
        for c, sp in cands[1:]:
            if c is None:  # the heuristic tile at an explicit split-K depth (WGRAD)
                assert mode == "wgrad" and sp >= 1
                continue
            bp, bq, bk, ns, halo = _decode(c)
            if halo and mode != "wgrad":
                assert bk == 32 and Fn.halo_eligible(g, bq, ns)
            if halo and mode == "wgrad":
                assert (bp, bq) == (64, 288) and sp >= 1
    # stride 2 / 1x1: no halo candidates, and the reduction must divide BK
    g2 = ConvGeom(G=1, N=4, H=16, W=16, C=96, K=128, R=1, S=1, stride=2, pad=0)
    for mode in ("fwd", "dgrad", "wgrad"):
        for c, _ in autotune.candidates(mode, g2)[1:]:
            if c is None:
                continue
            bp, bq, bk, ns, halo = _decode(c)
            assert not halo
            if mode == "fwd":
                assert g2.C % bk == 0
            if mode == "dgrad":
                assert g2.K % bk == 0
    # non-accumulating WGRAD cannot split-K: only the heuristic
    assert autotune.candidates("wgrad", g, accumulate=False) == [(None, 0)]


def test_halo_wgrad_eligibility_mirror():
    ok = ConvGeom(G=1, N=2, H=16, W=16, C=32, K=64, R=3, S=3, stride=1, pad=1)
    assert autotune.wgrad_halo_eligible(ok)
    for bad in (ConvGeom(1, 2, 16, 16, 32, 96, 3, 3, 1, 1),   # K % 64
                ConvGeom(1, 2, 4, 4, 32, 64, 3, 3, 1, 1),     # W = 4
                ConvGeom(1, 2, 56, 56, 32, 64, 3, 3, 1, 1),   # W = 56
                ConvGeom(1, 2, 16, 16, 32, 64, 3, 3, 2, 1)):  # stride 2
        assert not autotune.wgrad_halo_eligible(bad)


def test_pick_caches_and_respects_disable(monkeypatch):
    g = ConvGeom(G=1, N=2, H=8, W=8, C=32, K=32, R=3, S=3, stride=1, pad=1)
    monkeypatch.setattr(autotune, "ENABLED", False)
    calls = []
    assert autotune.pick("fwd", g, (False,), lambda c, s: calls.append(c)) == (None, 0)
    assert not calls
    monkeypatch.setitem(autotune._CACHE, autotune._key("fwd", g, (True,)), (123, 0))
    assert autotune.pick("fwd", g, (True,), lambda c, s: calls.append(c)) == (123, 0)


def test_fp32_plans_engine_choice():
    """fp32 conv plans: under "auto" a tuned plan carries its engine (X6 bit in the launch cfg),
    an x6-only entry falls back to X6, and a fixed engine forces / clears the bit."""
    from ddl25spring_amd.ops import functional_f32 as F32
    from ddl25spring_amd.ops.functional import ConvGeom
    g = ConvGeom(3, 7, 8, 8, 16, 16, 3, 3, 1, 1)
    key = "fwd:3,7,8,8,16,16,3,3,1,1"
    old_math, old_tuned = F32.math(), F32._TUNED
    try:
        F32._TUNED = {f"auto:{key}": [64, 128, 4, "mfma32"], f"x6:dgrad:3,7,8,8,16,16,3,3,1,1": [128, 64, 2]}
        F32.set_math("auto")
        F32._PLANS.clear()
        # a halo-eligible geometry (stride-1 "same" 3x3, OW 8) takes the halo X6 kernel first
        cfg, split = F32.plan(F32.F_FWD, g)
        assert cfg & F32.HALO_BIT and cfg & F32.X6_BIT
        F32.set_halo(False)
        cfg, split = F32.plan(F32.F_FWD, g)
        assert (cfg, split) == (F32.cfg_of(64, 128), 4) and F32._cfg(cfg) & F32.X6_BIT == 0
        cfg, split = F32.plan(F32.F_DGRAD, g)
        assert (cfg, split) == (F32.cfg_of(128, 64) | F32.X6_BIT, 2)
        F32.set_math("mfma32")
        assert F32._cfg(F32.cfg_of(64, 64) | F32.X6_BIT) == F32.cfg_of(64, 64)
        F32.set_math("x6")
        assert F32._cfg(F32.cfg_of(64, 64)) & F32.X6_BIT
    finally:
        F32._TUNED = old_tuned
        F32.set_math(old_math)
        F32.set_halo(True)
        F32._PLANS.clear()


def test_flat1x1_launch_geometry(monkeypatch):
    """Stride-1 1x1 convs re-shaped as rows of 128 pixels (opt-in DDL_F32_FLAT1X1): only eligible
    geometries change, the pixel count is preserved, and per-mode selection is honoured."""
    from ddl25spring_amd.ops import functional_f32 as F32
    monkeypatch.setattr(F32, "FLAT1X1", [True, "fdw"])
    g = ConvGeom(G=2, N=4, H=56, W=56, C=64, K=256, R=1, S=1, stride=1, pad=0)
    f = F32._launch_geom(g, "w")
    assert (f.G, f.N, f.W, f.C, f.K, f.R, f.stride, f.pad) == (2, 1, 128, 64, 256, 1, 1, 0)
    assert f.H * f.W == g.N * g.H * g.W and (f.P, f.Q) == (f.H, f.W)
    for keep in (ConvGeom(2, 4, 56, 56, 64, 256, 3, 3, 1, 1),   # 3x3
                 ConvGeom(2, 4, 56, 56, 64, 256, 1, 1, 2, 0),   # stride 2
                 ConvGeom(2, 4, 32, 32, 64, 256, 1, 1, 1, 0),   # power-of-two width: halo takes it as is
                 ConvGeom(2, 3, 7, 7, 64, 256, 1, 1, 1, 0)):    # 147 pixels: not a multiple of 128
        assert F32._launch_geom(keep, "f") is keep
    monkeypatch.setattr(F32, "FLAT1X1", [True, "d"])
    assert F32._launch_geom(g, "w") is g and F32._launch_geom(g, "d") != g
    monkeypatch.setattr(F32, "FLAT1X1", [False, "fdw"])
    assert F32._launch_geom(g, "d") is g


def test_fp32_measured_halo_and_vendor_entries(monkeypatch):
    """'x6h:' table entries set the halo plan (unless TARGET_WG = 1 pins split-K off), and 'blas:'
    entries route one product of a plain-GEMM linear to the vendor fp32 GEMM only as an opt-in
    (DDL_F32_BLAS=auto; the default 0 never does, 1 always)."""
    from ddl25spring_amd.ops import functional_f32 as F32
    from ddl25spring_amd.ops.functional import ConvGeom
    g = ConvGeom(3, 7, 8, 8, 16, 16, 3, 3, 1, 1)
    lin = ConvGeom(1, 64, 1, 1, 32, 48, 1, 1, 1, 0)
    old_math, old_tuned = F32.math(), F32._TUNED
    try:
        F32._TUNED = {"x6h:fwd:3,7,8,8,16,16,3,3,1,1": [64, 128, 2],
                      "blas:dgrad:1,64,1,1,32,48,1,1,1,0": [0.01, 0.02]}
        F32.set_math("auto")
        F32._PLANS.clear()
        assert F32.plan(F32.F_FWD, g) == (F32.cfg_of(64, 128) | F32.X6_BIT | F32.HALO_BIT, 2)
        monkeypatch.setattr(F32, "TARGET_WG", 1)
        F32._PLANS.clear()
        assert F32.plan(F32.F_FWD, g)[1] == 1
        assert not F32.vendor_gemm(F32.F_DGRAD, lin)  # default DDL_F32_BLAS=0: never the vendor GEMM
        monkeypatch.setattr(F32, "BLAS", ["auto"])
        assert F32.vendor_gemm(F32.F_DGRAD, lin) and not F32.vendor_gemm(F32.F_FWD, lin)
        monkeypatch.setattr(F32, "BLAS", ["0"])
        assert not F32.vendor_gemm(F32.F_DGRAD, lin)
        monkeypatch.setattr(F32, "BLAS", ["1"])
        assert F32.vendor_gemm(F32.F_FWD, lin)
    finally:
        F32._TUNED = old_tuned
        F32.set_math(old_math)
        F32._PLANS.clear()


def test_fp32_launch_record(tmp_path):
    """DDL_F32_RECORD=<file>: the (mode, geometry) pairs a process planned are written at exit, in
    the form scripts/conv_f32_tune.py --geoms-file reads."""
    import json
    import os
    import subprocess
    import sys
    from pathlib import Path
    out = tmp_path / "rec.json"
    code = ("from ddl25spring_amd.ops import functional_f32 as F32\n"
            "from ddl25spring_amd.ops.functional import ConvGeom\n"
            "g = ConvGeom(2, 4, 8, 8, 32, 64, 3, 3, 2, 1)\n"
            "F32.plan(F32.F_FWD, g); F32.plan(F32.F_WGRAD, g); F32.plan(F32.F_FWD, g)\n")
    subprocess.run([sys.executable, "-c", code], env=dict(os.environ, DDL_F32_RECORD=str(out)), check=True,
                   cwd=str(Path(__file__).resolve().parent.parent), timeout=120)
    rec = json.loads(out.read_text())
    assert rec == [{"mode": "fwd", "geom": [2, 4, 8, 8, 32, 64, 3, 3, 2, 1]},
                   {"mode": "wgrad", "geom": [2, 4, 8, 8, 32, 64, 3, 3, 2, 1]}]
