"""Halo-staged X6 fp32 convolution (csrc/kernels/conv_x6h.hip): FWD and stride-1 DGRAD against a
float64 PyTorch oracle, every fused epilogue, every tile geometry class (rows of one image, whole
images per tile, a partial last tile) and split-K; plus bitwise run-to-run determinism.

The reference's convs are stock fp32 nn.Conv2d (lab/tutorial_1a/hfl_complete.py:43-53); the
tolerance is the fp32 one of tests/test_fp32_gpu.py (1e-5 of the result's max-abs).
"""
import pytest
import torch

from ddl25spring_amd.ops import functional as Fn
from ddl25spring_amd.ops import functional_f32 as F32
from ddl25spring_amd.ops.functional import ConvGeom

from test_fp32_gpu import _close, _weights, ref_dgrad, ref_fwd

pytestmark = pytest.mark.gpu

GEOMS = [
    ConvGeom(G=2, N=5, H=32, W=32, C=64, K=64, R=3, S=3, stride=1, pad=1),    # 4 rows of one image
    ConvGeom(G=1, N=3, H=16, W=16, C=128, K=128, R=3, S=3, stride=1, pad=1),  # 8 rows
    ConvGeom(G=2, N=5, H=8, W=8, C=256, K=256, R=3, S=3, stride=1, pad=1),    # 2 images, partial tile
    ConvGeom(G=1, N=11, H=4, W=4, C=512, K=192, R=3, S=3, stride=1, pad=1),   # 8 images (explicit plan)
    ConvGeom(G=2, N=3, H=32, W=32, C=32, K=64, R=1, S=1, stride=1, pad=0),    # 1x1 (the im2col stem)
    ConvGeom(G=1, N=2, H=8, W=8, C=48, K=36, R=3, S=3, stride=1, pad=1),      # odd channel counts
    ConvGeom(G=1, N=2, H=64, W=64, C=32, K=32, R=3, S=3, stride=1, pad=1),    # 64 wide: 264-pixel halo
    ConvGeom(G=2, N=3, H=8, W=4, C=64, K=64, R=3, S=3, stride=1, pad=1),      # 4 wide, 8 tall
    # widths that are not a power of two: rows padded to one (PADW instances, split-K declined)
    ConvGeom(G=2, N=2, H=28, W=28, C=64, K=64, R=3, S=3, stride=1, pad=1),    # ResNet-50 stage 2 width
    ConvGeom(G=1, N=2, H=56, W=56, C=32, K=48, R=3, S=3, stride=1, pad=1),    # stage 1 width, 264-px halo
    ConvGeom(G=2, N=3, H=20, W=20, C=48, K=64, R=1, S=1, stride=1, pad=0),    # 1x1, partial last tile
]
IDS = [f"{g.C}x{g.K}_{g.H}x{g.W}_{g.R}n{g.N}" for g in GEOMS]


@pytest.fixture(autouse=True)
def _x6():
    old = F32.math()
    F32.set_math("x6")
    yield
    F32.set_math(old)


def _pin(mode, g, split):
    Pd = g.K if mode == F32.F_FWD else g.C
    F32.set_plan(mode, g, 128 if Pd > 64 else 64, 128, split, "x6h")


def _padded(g):
    return g.Q & (g.Q - 1) != 0


@pytest.mark.parametrize("split", [1, 2])
@pytest.mark.parametrize("geom", GEOMS, ids=IDS)
def test_x6h_fwd(cuda, geom, split):
    if geom.C % 16:
        pytest.skip("halo FWD needs C % 16 == 0")
    if split > 1 and _padded(geom):
        pytest.skip("row-padded tiles are never split over K")
    assert F32.halo_ok(F32.F_FWD, geom)
    _pin(F32.F_FWD, geom, split)
    try:
        torch.manual_seed(0)
        x = torch.randn(geom.G, geom.N, geom.H, geom.W, geom.C, device=cuda)
        w = _weights(geom, cuda)
        st = F32.SlotStats()
        y = Fn.conv_fwd(x, w, geom, stats=st)
        yr = ref_fwd(x.cpu(), w.cpu(), geom)
        _close(y, yr)
        t = st.t.double().cpu()
        yf = yr.reshape(geom.G, -1, geom.K)
        rows = st.rows
        assert rows == F32.slot_rows(F32.F_FWD, geom) and t.shape[1] == -(-yf.shape[1] // rows)
        assert rows == (128 if not _padded(geom) else 128 // (1 << (geom.Q - 1).bit_length()) * geom.Q)
        for i in range(t.shape[1]):
            blk = yf[:, i * rows:(i + 1) * rows]
            _close(t[:, i, 0], blk.sum(1))
            _close(t[:, i, 1], ((blk - blk.mean(1, keepdim=True)) ** 2).sum(1))
        bias = torch.randn(geom.G, geom.K, device=cuda)
        res = torch.randn(geom.G, geom.N, geom.P, geom.Q, geom.K, device=cuda)
        y2 = Fn.conv_fwd(x, w, geom, bias=bias, relu=True, residual=res)
        _close(y2, (yr + bias.cpu().double()[:, None, None, None] + res.cpu().double()).clamp_min(0))
        sc = torch.rand(geom.G, geom.C, device=cuda) + 0.5
        sh = torch.randn(geom.G, geom.C, device=cuda) * 0.3
        y3 = Fn.conv_fwd(x, w, geom, in_bn=(sc, sh))
        xa = (x.double() * sc.double()[:, None, None, None] + sh.double()[:, None, None, None]).clamp_min(0)
        _close(y3, ref_fwd(xa.cpu(), w.cpu(), geom))
        # bitwise run-to-run
        assert torch.equal(Fn.conv_fwd(x, w, geom, in_bn=(sc, sh)), y3)
    finally:
        F32.clear_plan(F32.F_FWD, geom)


@pytest.mark.parametrize("split", [1, 2])
@pytest.mark.parametrize("geom", GEOMS, ids=IDS)
def test_x6h_dgrad(cuda, geom, split):
    if geom.K % 16:
        pytest.skip("halo DGRAD needs K % 16 == 0")
    if split > 1 and _padded(geom):
        pytest.skip("row-padded tiles are never split over K")
    assert F32.halo_ok(F32.F_DGRAD, geom)
    _pin(F32.F_DGRAD, geom, split)
    try:
        torch.manual_seed(1)
        dy = torch.randn(geom.G, geom.N, geom.P, geom.Q, geom.K, device=cuda)
        w = _weights(geom, cuda)
        dxr = ref_dgrad(dy.cpu(), w.cpu(), geom)
        d1 = Fn.conv_dgrad(dy, w, geom)
        _close(d1, dxr)
        res = torch.randn(geom.G, geom.N, geom.H, geom.W, geom.C, device=cuda)
        mask = torch.randn(geom.G, geom.N, geom.H, geom.W, geom.C, device=cuda)
        d2 = Fn.conv_dgrad(dy, w, geom, residual=res, mask=mask)
        _close(d2, (dxr + res.cpu().double()) * (mask.cpu() > 0))
        # compact-grid residual (a stride-2 shortcut's dX, added on even pixels only)
        rc = torch.randn(geom.G, geom.N, (geom.H + 1) // 2, (geom.W + 1) // 2, geom.C, device=cuda)
        d2c = Fn.conv_dgrad(dy, w, geom, residual=rc, residual_sub=2)
        up = torch.zeros(geom.G, geom.N, geom.H, geom.W, geom.C, dtype=torch.float64)
        up[:, :, ::2, ::2] = rc.cpu().double()
        _close(d2c, dxr + up)
        bx = torch.randn(geom.G, geom.N, geom.H, geom.W, geom.C, device=cuda)
        mean = torch.randn(geom.G, geom.C, device=cuda) * 0.1
        rstd = torch.rand(geom.G, geom.C, device=cuda) + 0.5
        sc = torch.rand(geom.G, geom.C, device=cuda) + 0.5
        sh = torch.randn(geom.G, geom.C, device=cuda) * 0.2
        d3, part = Fn.conv_dgrad(dy, w, geom, bn=(bx, mean, rstd), mask_bn=(sc, sh))
        b = lambda t: t.cpu().double()[:, None, None, None]  # noqa: E731
        keep = (bx.cpu().double() * b(sc) + b(sh)) > 0
        want = dxr * keep
        _close(d3, want)
        xhat = (bx.cpu().double() - b(mean)) * b(rstd)
        p = part.double().cpu().sum(1)
        _close(p[:, 0], want.sum((1, 2, 3)))
        _close(p[:, 1], (want * xhat).sum((1, 2, 3)))
        assert torch.equal(Fn.conv_dgrad(dy, w, geom), d1)
    finally:
        F32.clear_plan(F32.F_DGRAD, geom)


@pytest.mark.parametrize("split", [1, 2])
@pytest.mark.parametrize("geom", GEOMS, ids=IDS)
def test_x6h_dgrad_bn_backward_operand(cuda, geom, split):
    """dy_bn: the DGRAD's dY operand is the following BN's backward A * dy + B * x_bn + C, applied
    as the halo is staged, and written out exactly once per element (the layer's WGRAD operand);
    the same call on a non-halo plan materialises it first (fallback)."""
    if geom.K % 16:
        pytest.skip("halo DGRAD needs K % 16 == 0")
    if split > 1 and _padded(geom):
        pytest.skip("row-padded tiles are never split over K")
    torch.manual_seed(2)
    dy = torch.randn(geom.G, geom.N, geom.P, geom.Q, geom.K, device=cuda)
    xb = torch.randn_like(dy)
    coef = torch.randn(geom.G, 3, geom.K, device=cuda)
    w = _weights(geom, cuda)
    c = coef.cpu().double()
    dc_ref = c[:, 0, None, None, None] * dy.cpu().double() + c[:, 1, None, None, None] * xb.cpu().double() \
        + c[:, 2, None, None, None]
    dxr = ref_dgrad(dc_ref, w.cpu(), geom)
    outs = []
    for engine in ("x6h", "x6"):
        Pd = geom.C
        F32.set_plan(F32.F_DGRAD, geom, 128 if Pd > 64 else 64, 128 if engine == "x6h" else 64, split, engine)
        try:
            assert F32.uses_halo(F32.F_DGRAD, geom) == (engine == "x6h")
            dc = torch.full_like(dy, float("nan"))
            dx = Fn.conv_dgrad(dy, w, geom, dy_bn=(xb, coef), dy_bn_out=dc)
            _close(dc, dc_ref, rel=1e-6)
            _close(dx, dxr)
            outs.append(dc)
        finally:
            F32.clear_plan(F32.F_DGRAD, geom)


WGEOMS = [
    ConvGeom(G=2, N=5, H=32, W=32, C=64, K=64, R=3, S=3, stride=1, pad=1),    # 4 rows per tile
    ConvGeom(G=1, N=3, H=16, W=16, C=128, K=128, R=3, S=3, stride=1, pad=1),  # 8 rows
    ConvGeom(G=2, N=5, H=8, W=8, C=256, K=64, R=3, S=3, stride=1, pad=1),     # 2 images per tile, partial
    ConvGeom(G=2, N=3, H=32, W=32, C=32, K=64, R=1, S=1, stride=1, pad=0),    # 1x1
]


@pytest.mark.parametrize("split", [0, 1])
@pytest.mark.parametrize("geom", WGEOMS, ids=[f"{g.C}x{g.K}_{g.H}x{g.W}_{g.R}n{g.N}" for g in WGEOMS])
def test_x6hw_wgrad(cuda, geom, split):
    """conv_x6hw.hip: halo-staged WGRAD (pixel-reduction MFMAs over a once-split X halo image) vs
    float64, plain and with the operand-side BN + ReLU of X, accumulating with a gscale (direct SGD),
    split over pixel tiles (0 = planner) or not; and bitwise repeatable."""
    from test_fp32_gpu import ref_wgrad
    old = F32.HALO_WGRAD[0], F32.HW_MIN_W
    F32.HALO_WGRAD[0], F32.HW_MIN_W = True, 0  # every geometry the kernel takes (8x8 included)
    try:
        _x6hw_case(cuda, geom, split, ref_wgrad)
    finally:
        F32.HALO_WGRAD[0], F32.HW_MIN_W = old


def _x6hw_case(cuda, geom, split, ref_wgrad):
    a = F32._args(geom)
    assert _lib_ok(a), "geometry must take the halo WGRAD"
    torch.manual_seed(3)
    x = torch.randn(geom.G, geom.N, geom.H, geom.W, geom.C, device=cuda)
    dy = torch.randn(geom.G, geom.N, geom.P, geom.Q, geom.K, device=cuda)
    dw = torch.zeros(geom.G, geom.K, geom.R, geom.S, geom.C, device=cuda)
    F32.conv_wgrad(dy, x, geom, dw, accumulate=False, split_k=split)
    ref = ref_wgrad(dy.cpu(), x.cpu(), geom)
    _close(dw, ref)
    dw2 = torch.zeros_like(dw)
    F32.conv_wgrad(dy, x, geom, dw2, accumulate=False, split_k=split)
    assert torch.equal(dw, dw2)
    sc = torch.rand(geom.G, geom.C, device=cuda) + 0.5
    sh = torch.randn(geom.G, geom.C, device=cuda) * 0.3
    xa = torch.relu(x.cpu().double() * sc.cpu().double()[:, None, None, None] + sh.cpu().double()[:, None, None, None])
    w0 = torch.randn_like(dw)
    w = w0.clone()
    F32.conv_wgrad(dy, x, geom, w, accumulate=True, gscale=-0.5, in_bn=(sc, sh), split_k=split)
    _close(w, w0.cpu().double() - 0.5 * ref_wgrad(dy.cpu(), xa, geom))


def _lib_ok(a):
    import ctypes
    from ddl25spring_amd.ops import _lib
    return bool(_lib.kernels().ddl_x6hw_ok(ctypes.byref(a)))


def test_x6h_split_weights(cuda):
    """The pre-split weight image reconstructs the fp32 weights exactly (h + m + l == w): per
    16-channel chunk three bf16 planes [h0..h15 | m0..m15 | l0..l15]."""
    g = ConvGeom(G=2, N=1, H=8, W=8, C=32, K=48, R=3, S=3, stride=1, pad=1)
    w = _weights(g, cuda)
    a = F32._args(g, w=w.data_ptr(), w_gs=w.stride(0))
    for mode in (F32.F_FWD, F32.F_DGRAD):
        img = F32.split_weights(a, mode, g, cuda)
        torch.cuda.synchronize()
        planes = img.view(torch.int16).view(g.G, -1, 3, 16)
        bf = lambda t: (t.to(torch.int32) << 16).view(torch.float32).double()  # noqa: E731
        rec = (bf(planes[:, :, 0]) + bf(planes[:, :, 1]) + bf(planes[:, :, 2])).reshape(g.G, -1)
        want = w if mode == F32.F_FWD else w.permute(0, 4, 2, 3, 1)  # DGRAD: [G][C][R][S][K]
        assert torch.equal(rec, want.reshape(g.G, -1).double())


def test_split_workspace_capture(cuda):
    """A split-K launch first requested inside a graph capture raises (no silent split-1 fallback);
    after ensure_workspace the captured launch equals the eager one bit for bit."""
    g = ConvGeom(G=1, N=3, H=4, W=4, C=512, K=512, R=3, S=3, stride=1, pad=1)
    _pin(F32.F_FWD, g, 4)
    try:
        x = torch.randn(g.G, g.N, g.H, g.W, g.C, device=cuda)
        w = _weights(g, cuda)
        saved = dict(F32._WS)
        F32._WS.clear()
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            graph = torch.cuda.CUDAGraph()
            with pytest.raises(RuntimeError, match="graph capture"):
                with torch.cuda.graph(graph, stream=s):
                    Fn.conv_fwd(x, w, g)
        torch.cuda.synchronize()
        F32._WS.update(saved)
        F32.ensure_workspace(cuda)
        eager = Fn.conv_fwd(x, w, g)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            y = Fn.conv_fwd(x, w, g)
        graph.replay()
        torch.cuda.synchronize()
        assert torch.equal(y, eager)
    finally:
        F32.clear_plan(F32.F_FWD, g)


def test_gram_blocked_k129(cuda):
    """Krum's Gram for K > 128 clients: blocked native Grams, float64-close and bit-reproducible."""
    X = torch.randn(129, 4096, device=cuda)
    G1 = Fn.gram(X)
    ref = (X.double() @ X.double().t()).cpu()
    _close(G1, ref)
    assert torch.equal(Fn.gram(X), G1)


NET = [ConvGeom(G=2, N=16, H=h, W=h, C=c, K=c, R=3, S=3, stride=1, pad=1) for h, c in
       ((32, 64), (16, 128), (8, 256), (4, 512))] + [ConvGeom(G=2, N=16, H=32, W=32, C=32, K=64, R=1, S=1, stride=1,
                                                               pad=0)]


@pytest.mark.parametrize("geom", NET, ids=[f"c{g.C}k{g.K}_{g.H}_r{g.R}" for g in NET])
def test_x6h_network_shapes_auto_plan(cuda, geom):
    """The ResNet-18 (CIFAR) stride-1 layers at a small batch with the DEFAULT plan (halo where
    eligible, its split-K choice) and the fused epilogues the network uses together: FWD with
    operand-side BN + statistics; DGRAD with residual + ReLU mask + the producer BN's reduce, and
    with the recomputed-mask BN reduce. Run twice: bitwise equal."""
    torch.manual_seed(5)
    x = torch.randn(geom.G, geom.N, geom.H, geom.W, geom.C, device=cuda)
    w = _weights(geom, cuda)
    sc = torch.rand(geom.G, geom.C, device=cuda) + 0.5
    sh = torch.randn(geom.G, geom.C, device=cuda) * 0.3
    st = F32.SlotStats()
    y = Fn.conv_fwd(x, w, geom, stats=st, in_bn=(sc, sh))
    xa = (x.double() * sc.double()[:, None, None, None] + sh.double()[:, None, None, None]).clamp_min(0)
    yr = ref_fwd(xa.cpu(), w.cpu(), geom)
    _close(y, yr)
    tot = st.t.double().cpu()[:, :, 0].sum(1)
    _close(tot, yr.reshape(geom.G, -1, geom.K).sum(1))
    st2 = F32.SlotStats()
    assert torch.equal(Fn.conv_fwd(x, w, geom, stats=st2, in_bn=(sc, sh)), y) and torch.equal(st2.t, st.t)
    if geom.R == 1:
        return
    dy = torch.randn(geom.G, geom.N, geom.P, geom.Q, geom.K, device=cuda)
    dxr = ref_dgrad(dy.cpu(), w.cpu(), geom)
    res = torch.randn(geom.G, geom.N, geom.H, geom.W, geom.C, device=cuda)
    mask = torch.randn(geom.G, geom.N, geom.H, geom.W, geom.C, device=cuda)
    bx = torch.randn(geom.G, geom.N, geom.H, geom.W, geom.C, device=cuda)
    mean = torch.randn(geom.G, geom.C, device=cuda) * 0.1
    rstd = torch.rand(geom.G, geom.C, device=cuda) + 0.5
    d1, part = Fn.conv_dgrad(dy, w, geom, residual=res, mask=mask, bn=(bx, mean, rstd))
    want = (dxr + res.cpu().double()) * (mask.cpu() > 0)
    _close(d1, want)
    b = lambda t: t.cpu().double()[:, None, None, None]  # noqa: E731
    xhat = (bx.cpu().double() - b(mean)) * b(rstd)
    p = part.double().cpu().sum(1)
    _close(p[:, 0], want.sum((1, 2, 3)))
    _close(p[:, 1], (want * xhat).sum((1, 2, 3)))
    d1b, part_b = Fn.conv_dgrad(dy, w, geom, residual=res, mask=mask, bn=(bx, mean, rstd))
    assert torch.equal(d1b, d1) and torch.equal(part_b, part)
    sc2 = torch.rand(geom.G, geom.C, device=cuda) + 0.5
    sh2 = torch.randn(geom.G, geom.C, device=cuda) * 0.2
    d2, part2 = Fn.conv_dgrad(dy, w, geom, bn=(bx, mean, rstd), mask_bn=(sc2, sh2))
    keep = (bx.cpu().double() * b(sc2) + b(sh2)) > 0
    _close(d2, dxr * keep)


@pytest.mark.parametrize("side", [False, True])
def test_presplit_scope_matches_per_launch(cuda, monkeypatch, side):
    """PresplitScope (Net.train_step): the first pass records the halo launches' weight images,
    later passes read the images ONE multi-tensor launch made at scope entry (side: the first
    image up front, the rest on a side stream the step's stream joins at their first use) —
    bitwise the per-launch split's results, refreshed when the weights change between steps."""
    monkeypatch.setattr(F32, "PRESPLIT_SIDE", [side])
    geoms = [ConvGeom(G=2, N=3, H=16, W=16, C=64, K=128, R=3, S=3, stride=1, pad=1),
             ConvGeom(G=2, N=3, H=16, W=16, C=128, K=128, R=1, S=1, stride=1, pad=0)]
    torch.manual_seed(7)
    xs = [torch.randn(g.G, g.N, g.H, g.W, g.C, device=cuda) for g in geoms]
    dys = [torch.randn(g.G, g.N, g.P, g.Q, g.K, device=cuda) for g in geoms]
    ws = [_weights(g, cuda) for g in geoms]
    for g in geoms:
        _pin(F32.F_FWD, g, 1)
        _pin(F32.F_DGRAD, g, 1)

    def run():
        return [t for g, x, dy, w in zip(geoms, xs, dys, ws)
                for t in (Fn.conv_fwd(x, w, g), Fn.conv_dgrad(dy, w, g))]

    try:
        plain = run()
        scope = F32.PresplitScope()
        with scope:
            rec = run()
        assert scope.state == "ready" and len(scope.keys) == 4
        assert len(scope.tables) == (2 if side else 1) and len(scope.tail) == (3 if side else 0)
        with scope:
            pre = run()
        for a, b, c in zip(plain, rec, pre):
            assert torch.equal(a, b) and torch.equal(a, c)
        for w in ws:
            w.mul_(1.01)
        plain2 = run()
        with scope:
            pre2 = run()
        for a, b in zip(plain2, pre2):
            assert torch.equal(a, b)
    finally:
        for g in geoms:
            F32.clear_plan(F32.F_FWD, g)
            F32.clear_plan(F32.F_DGRAD, g)
