"""Numerics of every HIP kernel against the plain-PyTorch fp32 reference of the same op."""
import pytest
import torch

from ddl25spring_amd.ops import functional as Fn
from ddl25spring_amd.ops import reference as ref
from ddl25spring_amd.ops.functional import ConvGeom

pytestmark = pytest.mark.gpu


def _close(a, b, rel=2e-2, abs_=1e-3):
    a = a.float().cpu()
    b = b.float().cpu()
    scale = b.abs().max().item() + 1e-6
    err = (a - b).abs().max().item()
    assert err <= rel * scale + abs_, f"max err {err} vs scale {scale}"


def _rand(*shape, dev="cpu", scale=1.0):
    return (torch.randn(*shape) * scale).to(torch.bfloat16).to(dev)


GEOMS = [
    ConvGeom(G=2, N=3, H=8, W=8, C=32, K=64, R=3, S=3, stride=1, pad=1),
    ConvGeom(G=1, N=2, H=9, W=9, C=64, K=128, R=3, S=3, stride=2, pad=1),
    ConvGeom(G=3, N=4, H=4, W=4, C=128, K=64, R=1, S=1, stride=2, pad=0),
    ConvGeom(G=2, N=37, H=1, W=1, C=96, K=32, R=1, S=1, stride=1, pad=0),
    ConvGeom(G=1, N=2, H=26, W=26, C=32, K=64, R=3, S=3, stride=1, pad=0),
    ConvGeom(G=2, N=4, H=8, W=8, C=256, K=256, R=3, S=3, stride=1, pad=1),
    ConvGeom(G=2, N=3, H=7, W=5, C=64, K=64, R=3, S=3, stride=2, pad=1),   # odd sizes, phased dgrad
    ConvGeom(G=1, N=2, H=5, W=6, C=32, K=64, R=1, S=1, stride=2, pad=0),   # 1x1/2: empty phases
    ConvGeom(G=1, N=2, H=9, W=9, C=32, K=32, R=3, S=3, stride=3, pad=1),   # stride 3 (unphased)
    ConvGeom(G=1, N=2, H=16, W=16, C=32, K=64, R=7, S=7, stride=2, pad=3), # 7x7/2 stem shape
]


def _weights(geom, dev, strided=True):
    # strided group view into a flat [G, P] buffer, like the flat parameter store
    inner = geom.K * geom.R * geom.S * geom.C
    pad = 96 if strided else 0
    flat = _rand(geom.G, inner + pad, dev=dev, scale=0.1)
    return flat[:, :inner].view(geom.G, geom.K, geom.R, geom.S, geom.C) if not strided else \
        flat[:, 16:16 + inner].unflatten(1, (geom.K, geom.R, geom.S, geom.C))


@pytest.mark.parametrize("geom", GEOMS, ids=lambda g: f"{g.C}x{g.K}_{g.H}_{g.R}s{g.stride}p{g.pad}")
def test_conv_fwd(cuda, geom):
    x = _rand(geom.G, geom.N, geom.H, geom.W, geom.C, dev=cuda)
    w = _weights(geom, cuda)
    bias = torch.randn(geom.G, geom.K, device=cuda)
    stats = torch.zeros(geom.G, 2, geom.K, device=cuda)
    y = Fn.conv_fwd(x, w, geom, stats=stats)
    stats_ref = torch.zeros(geom.G, 2, geom.K)
    y_ref = ref.conv_fwd(x.cpu(), w.cpu(), geom, stats=stats_ref)
    _close(y, y_ref)
    _close(stats, stats_ref, rel=1e-3)
    y2 = Fn.conv_fwd(x, w, geom, bias=bias, relu=True)
    _close(y2, ref.conv_fwd(x.cpu(), w.cpu(), geom, bias=bias.cpu(), relu=True))


@pytest.mark.parametrize("geom", GEOMS, ids=lambda g: f"{g.C}x{g.K}_{g.H}_{g.R}s{g.stride}p{g.pad}")
def test_conv_dgrad(cuda, geom):
    dy = _rand(geom.G, geom.N, geom.P, geom.Q, geom.K, dev=cuda)
    w = _weights(geom, cuda)
    dx = Fn.conv_dgrad(dy, w, geom)
    _close(dx, ref.conv_dgrad(dy.cpu(), w.cpu(), geom))
    res = _rand(geom.G, geom.N, geom.H, geom.W, geom.C, dev=cuda)
    mask = _rand(geom.G, geom.N, geom.H, geom.W, geom.C, dev=cuda)
    dx2 = Fn.conv_dgrad(dy, w, geom, residual=res, mask=mask)
    _close(dx2, ref.conv_dgrad(dy.cpu(), w.cpu(), geom, residual=res.cpu(), mask=mask.cpu()))


@pytest.mark.parametrize("geom", GEOMS, ids=lambda g: f"{g.C}x{g.K}_{g.H}_{g.R}s{g.stride}p{g.pad}")
def test_conv_wgrad(cuda, geom):
    x = _rand(geom.G, geom.N, geom.H, geom.W, geom.C, dev=cuda)
    dy = _rand(geom.G, geom.N, geom.P, geom.Q, geom.K, dev=cuda)
    inner = geom.K * geom.R * geom.S * geom.C
    flat = torch.zeros(geom.G, inner + 64, device=cuda)
    dw = flat[:, 32:32 + inner].unflatten(1, (geom.K, geom.R, geom.S, geom.C))
    Fn.conv_wgrad(dy, x, geom, dw, accumulate=True)
    dw_ref = torch.zeros(geom.G, geom.K, geom.R, geom.S, geom.C)
    ref.conv_wgrad(dy.cpu(), x.cpu(), geom, dw_ref)
    _close(dw, dw_ref, rel=2e-3)
    assert flat[:, :32].abs().max().item() == 0 and flat[:, 32 + inner:].abs().max().item() == 0


def test_conv_tile_configs(cuda):
    geom = ConvGeom(G=2, N=3, H=8, W=8, C=128, K=128, R=3, S=3, stride=1, pad=1)
    x = _rand(geom.G, geom.N, geom.H, geom.W, geom.C, dev=cuda)
    w = _weights(geom, cuda)
    dy = _rand(geom.G, geom.N, geom.P, geom.Q, geom.K, dev=cuda)
    y_ref = ref.conv_fwd(x.cpu(), w.cpu(), geom)
    dx_ref = ref.conv_dgrad(dy.cpu(), w.cpu(), geom)
    dw_ref = torch.zeros(geom.G, geom.K, geom.R, geom.S, geom.C)
    ref.conv_wgrad(dy.cpu(), x.cpu(), geom, dw_ref)
    cfgs = Fn.CONV_TILES
    for bp, bq, bk, ns in cfgs:
        cfg = Fn.conv_cfg(bp, bq, bk, ns)
        _close(Fn.conv_fwd(x, w, geom, cfg=cfg), y_ref)
        _close(Fn.conv_dgrad(dy, w, geom, cfg=cfg), dx_ref)
        for splits in (1, 3):
            dw = torch.zeros(geom.G, geom.K, geom.R, geom.S, geom.C, device=cuda)
            Fn.conv_wgrad(dy, x, geom, dw, cfg=cfg, splits=splits)
            _close(dw, dw_ref, rel=2e-3)


HALO_GEOMS = [
    ConvGeom(G=2, N=3, H=32, W=32, C=64, K=64, R=3, S=3, stride=1, pad=1),    # layer-1 shape
    ConvGeom(G=1, N=2, H=16, W=16, C=96, K=160, R=3, S=3, stride=1, pad=1),   # odd block counts
    ConvGeom(G=2, N=3, H=8, W=8, C=256, K=128, R=3, S=3, stride=1, pad=1),    # 2 images per tile
    ConvGeom(G=1, N=5, H=8, W=8, C=64, K=64, R=3, S=3, stride=1, pad=1),      # partial last tile
    ConvGeom(G=1, N=4, H=4, W=32, C=32, K=64, R=3, S=3, stride=1, pad=1),     # 1 channel block
]


@pytest.mark.parametrize("geom", HALO_GEOMS, ids=lambda g: f"{g.C}x{g.K}_{g.H}x{g.W}")
def test_conv_halo(cuda, geom):
    """Halo-staged 3x3 stride-1 kernels (activation tile + halo DMA'd once per channel block)
    match the fp32 reference for every tile config the shape admits, with the fused epilogues."""
    g = geom
    x = _rand(g.G, g.N, g.H, g.W, g.C, dev=cuda)
    w = _weights(g, cuda)
    dy = _rand(g.G, g.N, g.P, g.Q, g.K, dev=cuda)
    bias = torch.randn(g.G, g.K, device=cuda)
    res = _rand(g.G, g.N, g.H, g.W, g.C, dev=cuda)
    mask = _rand(g.G, g.N, g.H, g.W, g.C, dev=cuda)
    st_ref = torch.zeros(g.G, 2, g.K)
    y_ref = ref.conv_fwd(x.cpu(), w.cpu(), g, bias=bias.cpu(), relu=True, stats=st_ref)
    dx_ref = ref.conv_dgrad(dy.cpu(), w.cpu(), g, residual=res.cpu(), mask=mask.cpu())
    ran = 0
    for bp, bq, ns in Fn.HALO_TILES:
        cfg = Fn.conv_cfg(bp, bq, 32, ns, halo=True)
        if not Fn.halo_eligible(g, bq, ns):
            with pytest.raises(RuntimeError):
                Fn.conv_fwd(x, w, g, cfg=cfg)
            continue
        ran += 1
        st = Fn.stats_buffer(g.G, g.K, cuda)
        _close(Fn.conv_fwd(x, w, g, bias=bias, relu=True, stats=st, cfg=cfg), y_ref)
        _close(st.sum(1), st_ref, rel=2e-3)
        _close(Fn.conv_dgrad(dy, w, g, residual=res, mask=mask, cfg=cfg), dx_ref)
    assert ran > 0
    # the automatic choice (halo where eligible) agrees too
    _close(Fn.conv_fwd(x, w, g, bias=bias, relu=True), y_ref)
    _close(Fn.conv_dgrad(dy, w, g, residual=res, mask=mask), dx_ref)


WGRAD_HALO_GEOMS = [
    ConvGeom(G=2, N=3, H=32, W=32, C=64, K=64, R=3, S=3, stride=1, pad=1),
    ConvGeom(G=1, N=2, H=16, W=16, C=96, K=128, R=3, S=3, stride=1, pad=1),
    ConvGeom(G=2, N=3, H=8, W=8, C=32, K=64, R=3, S=3, stride=1, pad=1),
    ConvGeom(G=1, N=2, H=4, W=32, C=64, K=192, R=3, S=3, stride=1, pad=1),
]


@pytest.mark.parametrize("geom", WGRAD_HALO_GEOMS, ids=lambda g: f"{g.C}x{g.K}_{g.H}x{g.W}")
def test_conv_wgrad_halo(cuda, geom):
    """Halo WGRAD (a 32-pixel K-step's rows + halo DMA'd once, 9 taps read shifted windows) ==
    the fp32 reference, for split-K counts 1, 3 and automatic, accumulating into a strided view."""
    g = geom
    x = _rand(g.G, g.N, g.H, g.W, g.C, dev=cuda)
    dy = _rand(g.G, g.N, g.P, g.Q, g.K, dev=cuda)
    dw_ref = torch.zeros(g.G, g.K, g.R, g.S, g.C)
    ref.conv_wgrad(dy.cpu(), x.cpu(), g, dw_ref)
    cfg = Fn.conv_cfg(64, 288, 32, 4, halo=True)
    inner = g.K * g.R * g.S * g.C
    for splits in (1, 3, 0):
        flat = torch.zeros(g.G, inner + 64, device=cuda)
        dw = flat[:, 32:32 + inner].unflatten(1, (g.K, g.R, g.S, g.C))
        Fn.conv_wgrad(dy, x, g, dw, accumulate=True, cfg=cfg, splits=splits)
        _close(dw, dw_ref, rel=2e-3)
        assert flat[:, :32].abs().max().item() == 0 and flat[:, 32 + inner:].abs().max().item() == 0
    with pytest.raises(RuntimeError):  # not eligible: stride 2
        g2 = ConvGeom(G=1, N=2, H=8, W=8, C=64, K=64, R=3, S=3, stride=2, pad=1)
        Fn.conv_wgrad(_rand(1, 2, 4, 4, 64, dev=cuda), _rand(1, 2, 8, 8, 64, dev=cuda), g2,
                      torch.zeros(1, 64, 3, 3, 64, device=cuda), cfg=cfg)


def test_batchnorm(cuda):
    G, N, H, W, C = 2, 5, 6, 6, 64
    x = _rand(G, N, H, W, C, dev=cuda, scale=2.0) + 0.5
    stats = torch.stack([x.float().reshape(G, -1, C).sum(1), (x.float() ** 2).reshape(G, -1, C).sum(1)], 1)
    gamma = torch.rand(G, C, device=cuda) + 0.5
    beta = torch.randn(G, C, device=cuda)
    rm, rv = torch.zeros(G, C, device=cuda), torch.ones(G, C, device=cuda)
    rm_r, rv_r = rm.cpu().clone(), rv.cpu().clone()
    M = N * H * W
    sc, sh, mu, rs = Fn.bn_finalize(stats, gamma, beta, rm, rv, M)
    sc_r, sh_r, mu_r, rs_r = ref.bn_finalize(stats.cpu(), gamma.cpu(), beta.cpu(), rm_r, rv_r, M, 1e-5, 0.1, True)
    _close(sc, sc_r, rel=1e-4); _close(sh, sh_r, rel=1e-4); _close(rm, rm_r, rel=1e-4); _close(rv, rv_r, rel=1e-4)
    r = _rand(G, N, H, W, C, dev=cuda)
    for act in (0, 1, 2):
        _close(Fn.bn_apply(x, sc, sh, r=r, rscale=sc, rshift=sh, act=act),
               ref.bn_apply(x.cpu(), sc_r, sh_r, r.cpu(), sc_r, sh_r, act))
    y = Fn.bn_apply(x, sc, sh, act=1)
    dy = _rand(G, N, H, W, C, dev=cuda)
    dg = torch.zeros(G, C, device=cuda); db = torch.zeros(G, C, device=cuda)
    sums = Fn.bn_bwd_reduce(dy, y, x, mu, rs, dg, db)
    dg_r = torch.zeros(G, C); db_r = torch.zeros(G, C)
    sums_r = ref.bn_bwd_reduce(dy.cpu(), y.cpu(), x.cpu(), mu_r, rs_r, dg_r, db_r)
    _close(sums, sums_r, rel=2e-3); _close(dg, dg_r, rel=2e-3); _close(db, db_r, rel=2e-3)
    dx, dym = Fn.bn_bwd_apply(dy, y, x, mu, rs, gamma, sums, emit_dym=True)
    dx_r, dym_r = ref.bn_bwd_apply(dy.cpu(), y.cpu(), x.cpu(), mu_r, rs_r, gamma.cpu(), sums_r, True)
    _close(dx, dx_r); _close(dym, dym_r)
    # fused three-launch backward == reduce + apply; striped statistics (conv epilogue format)
    dg2 = torch.zeros(G, C, device=cuda); db2 = torch.zeros(G, C, device=cuda)
    dx2, dym2 = Fn.bn_backward(dy, y, x, mu, rs, gamma, dg2, db2, emit_dym=True)
    _close(dx2, dx_r); _close(dym2, dym_r); _close(dg2, dg_r, rel=2e-3); _close(db2, db_r, rel=2e-3)
    st = Fn.bn_stats(x)
    assert st.shape == (G, Fn.BN_STRIPES, 2, C)
    _close(st.sum(1), stats.cpu(), rel=1e-3)
    sc2, sh2, _, _ = Fn.bn_finalize(st, gamma, beta, None, None, M)
    _close(sc2, sc_r, rel=1e-4); _close(sh2, sh_r, rel=1e-4)


def test_bn_reduce_wide_channels(cuda):
    """2048-channel reduces (ResNet-50's last stage): the grid is capped by the stripes' atomic
    budget, so each block sweeps many rows (4 in flight per thread). Sums == fp32 references."""
    G, N, H, W, C = 1, 4, 32, 32, 2048
    x = _rand(G, N, H, W, C, dev=cuda) + 0.3
    dy = _rand(G, N, H, W, C, dev=cuda)
    y = _rand(G, N, H, W, C, dev=cuda)
    xf = x.float().reshape(G, -1, C)
    st = Fn.bn_stats(x)
    _close(st.sum(1), torch.stack([xf.sum(1), (xf * xf).sum(1)], 1).cpu(), rel=1e-3)
    mu = torch.randn(G, C, device=cuda) * 0.1
    rs = torch.rand(G, C, device=cuda) + 0.5
    dg = torch.zeros(G, C, device=cuda); db = torch.zeros(G, C, device=cuda)
    sums = Fn.bn_bwd_reduce(dy, y, x, mu, rs, dg, db)
    dg_r = torch.zeros(G, C); db_r = torch.zeros(G, C)
    sums_r = ref.bn_bwd_reduce(dy.cpu(), y.cpu(), x.cpu(), mu.cpu(), rs.cpu(), dg_r, db_r)
    _close(sums, sums_r, rel=2e-3)
    # pool backward with the BN reduce at the same width
    dp = _rand(G, N, C, dev=cuda)
    dx, part = Fn.avgpool_bwd_bn(dp, x, (y, mu, rs))
    dx_r, part_r = Fn.avgpool_bwd_bn(dp.cpu(), x.cpu(), (y.cpu(), mu.cpu(), rs.cpu()))
    _close(dx, dx_r, rel=1e-2)
    _close(part.sum(1), part_r.sum(1), rel=2e-3)


def test_bn_dual_finalize_and_backward(cuda):
    """bn_finalize2 / bn_backward2 (a block's output BN and its shortcut's BN in one launch each)
    == the single-BN kernels, including the running statistics and d(gamma) / d(beta)."""
    G, N, H, W, C = 2, 3, 5, 6, 128
    M = N * H * W
    xs = [_rand(G, N, H, W, C, dev=cuda, scale=1.5) + 0.2 for _ in range(2)]
    bns = []
    for x in xs:
        st = Fn.bn_stats(x)
        bns.append([st, torch.rand(G, C, device=cuda) + 0.5, torch.randn(G, C, device=cuda),
                    torch.randn(G, C, device=cuda), torch.rand(G, C, device=cuda) + 0.5, M])
    copies = [[t.clone() if torch.is_tensor(t) else t for t in bn] for bn in bns]
    o1, o2 = Fn.bn_finalize2(bns[0], bns[1])
    for got, bn in zip((o1, o2), copies):
        want = Fn.bn_finalize(*bn)
        for a, b in zip(got, want):
            _close(a, b, rel=1e-5)
    for bn, cp in zip(bns, copies):  # running statistics updated identically
        _close(bn[3], cp[3], rel=1e-5); _close(bn[4], cp[4], rel=1e-5)
    dy = _rand(G, N, H, W, C, dev=cuda)
    args, ref_out = [], []
    for x, (sc, sh, mu, rs), bn in zip(xs, (o1, o2), bns):
        part = Fn.bn_bwd_reduce_part(dy, None, x, mu, rs)
        dg, db = torch.zeros(G, C, device=cuda), torch.zeros(G, C, device=cuda)
        dg2, db2 = dg.clone(), db.clone()
        args.append((x, mu, rs, bn[1], dg, db, part))
        ref_out.append((Fn.bn_backward(dy, None, x, mu, rs, bn[1], dg2, db2, part=part.clone()), dg2, db2))
    dxa, dxb = Fn.bn_backward2(dy, args[0], args[1])
    for dx, a, (rdx, rdg, rdb) in zip((dxa, dxb), args, ref_out):
        _close(dx, rdx, rel=1e-2)
        _close(a[4], rdg, rel=1e-4); _close(a[5], rdb, rel=1e-4)


def test_pools_act_dropout(cuda):
    x = _rand(2, 3, 8, 6, 64, dev=cuda)
    _close(Fn.maxpool2_fwd(x), ref.maxpool2_fwd(x.cpu()), rel=0, abs_=0)
    dy = _rand(2, 3, 4, 3, 64, dev=cuda)
    _close(Fn.maxpool2_bwd(x, dy), ref.maxpool2_bwd(x.cpu(), dy.cpu()), rel=0, abs_=0)
    # general k/s/p max-pool (ResNet-50 3x3/2 pad 1): recompute and saved-argmax backward
    for k_, s_, p_ in ((3, 2, 1), (2, 2, 0), (3, 1, 1)):
        y = Fn.maxpool_fwd(x, k_, s_, p_)
        y2, am = Fn.maxpool_fwd(x, k_, s_, p_, want_argmax=True)
        _close(y, Fn.maxpool_fwd(x.cpu(), k_, s_, p_), rel=0, abs_=0)
        assert torch.equal(y, y2)
        dyp = _rand(*y.shape, dev=cuda)
        want = Fn.maxpool_bwd(x.cpu(), dyp.cpu(), k_, s_, p_)
        _close(Fn.maxpool_bwd(x, dyp, k_, s_, p_), want)
        _close(Fn.maxpool_bwd(x, dyp, k_, s_, p_, argmax=am), want)
    _close(Fn.avgpool_fwd(x), ref.avgpool_fwd(x.cpu()))
    d2 = _rand(2, 3, 64, dev=cuda)
    _close(Fn.avgpool_bwd(d2, 8, 6), ref.avgpool_bwd(d2.cpu(), 8, 6))
    for act in (1, 2):
        y = Fn.act_fwd(x, act)
        _close(y, ref.act_fwd(x.cpu(), act))
        _close(Fn.act_bwd(y, x, act), ref.act_bwd(y.cpu(), x.cpu(), act))
    ones = torch.ones(64, 1024, dtype=torch.bfloat16, device=cuda)
    d = Fn.dropout(ones, 0.25, seed=7, offset=0)
    keep = (d.float() > 0).float().mean().item()
    assert abs(keep - 0.75) < 0.01
    assert torch.allclose(d.float()[d.float() > 0], torch.full_like(d.float()[d.float() > 0], 1 / 0.75), rtol=1e-2)
    d_again = Fn.dropout(ones, 0.25, seed=7, offset=0)
    assert torch.equal(d, d_again)
    out = torch.zeros(2, 64, device=cuda)
    Fn.channel_sum(x, out)
    _close(out, x.cpu().float().reshape(2, -1, 64).sum(1), rel=1e-3)


def test_cross_entropy(cuda):
    G, N, ld, ncls = 3, 50, 32, 10
    logits = _rand(G, N, ld, dev=cuda, scale=3)
    labels = torch.randint(0, ncls, (G, N), device=cuda)
    loss, d, corr = Fn.cross_entropy(logits, labels, ncls=ncls, scale=1 / N, with_correct=True)
    loss_r = torch.zeros(G); corr_r = torch.zeros(G, dtype=torch.int32)
    d_r = ref.ce_fwd_bwd(logits.cpu(), labels.cpu(), None, ncls, 1 / N, loss_r, corr_r)
    _close(loss, loss_r, rel=1e-4); _close(d, d_r); assert torch.equal(corr.cpu(), corr_r)
    # torch oracle
    lt = torch.stack([torch.nn.functional.cross_entropy(logits[g, :, :ncls].float().cpu(), labels[g].cpu()) for g in range(G)])
    _close(loss, lt, rel=1e-4)
    targets = torch.softmax(torch.randn(G, N, ncls), -1).to(cuda)
    loss2, d2, _ = Fn.cross_entropy(logits, targets=targets, ncls=ncls, scale=1 / N)
    loss2_r = torch.zeros(G)
    d2_r = ref.ce_fwd_bwd(logits.cpu(), None, targets.cpu(), ncls, 1 / N, loss2_r)
    _close(loss2, loss2_r, rel=1e-4); _close(d2, d2_r)


def test_optimizers(cuda):
    n = 1000 * 4 + 3
    p = torch.randn(n, device=cuda); g = torch.randn(n, device=cuda)
    for momentum, nest in ((0.0, False), (0.9, False), (0.9, True)):
        pc, mc = p.cpu().clone(), torch.zeros(n)
        pg, mg = p.clone(), torch.zeros(n, device=cuda)
        sh = torch.empty(n, dtype=torch.bfloat16, device=cuda)
        for step in range(3):
            Fn.sgd_step(pg, g, mg, sh, 0.1, 1e-4, momentum, 0.0, nest, step == 0)
            ref.sgd(pc, g.cpu(), mc, None, 0.1, 1e-4, momentum, 0.0, nest, step == 0)
        _close(pg, pc, rel=1e-5, abs_=1e-6)
        _close(sh, pc)
    # adam / adamw vs torch.optim
    for decoupled in (False, True):
        w = torch.nn.Parameter(p.cpu().clone())
        opt = (torch.optim.AdamW if decoupled else torch.optim.Adam)([w], lr=1e-2, weight_decay=0.01)
        pg = p.clone(); m = torch.zeros(n, device=cuda); v = torch.zeros(n, device=cuda)
        for step in range(1, 4):
            w.grad = g.cpu().clone(); opt.step()
            Fn.adam_step(pg, g, m, v, None, 1e-2, 0.9, 0.999, 1e-8, 0.01, step, decoupled)
        _close(pg, w.detach(), rel=1e-5, abs_=1e-6)


def test_aggregation(cuda):
    G, P = 5, 12345
    buf = torch.randn(G, P + 7, device=cuda)
    src = buf[:, :P]
    coeff = torch.rand(G, device=cuda)
    out = torch.empty(P, device=cuda)
    Fn.weighted_sum(src, coeff, out)
    _close(out, (coeff.cpu()[:, None] * src.cpu()).sum(0), rel=1e-5)
    dst = torch.zeros(G, P + 7, device=cuda)
    sh = torch.zeros(G, P + 7, dtype=torch.bfloat16, device=cuda)
    Fn.broadcast_rows(out, dst[:, :P], sh[:, :P])
    assert torch.equal(dst[:, :P], out.expand(G, P)) and dst[:, P:].abs().max() == 0
    for K in (3, 8, 20, 33, 64, 65, 100, 128):
        X = torch.randn(K, 20000, device=cuda)
        c = torch.randn(20000, device=cuda)
        _close(Fn.gram(X, c), ref.gram(X.cpu().double(), c.cpu().double()).float(), rel=1e-5)
        for mode, trim in (("median", 0), ("trimmed", K // 4)):
            if mode == "trimmed" and K - 2 * trim < 1:
                continue
            _close(Fn.coord_select(X, mode, trim), ref.coord_select(X.cpu(), 0 if mode == "median" else 1, trim), rel=1e-6)


def test_robust_kernels_deterministic_and_bounded(cuda):
    """The Gram sums per-block partials in a fixed order (no float atomics): bit-identical across
    calls, so Krum's argsort never flips between runs. K > 128: the Gram is assembled from native
    row-block Grams (still fixed-order, bit-reproducible); coordinate selection raises instead of
    falling back."""
    X = torch.randn(100, 300_000, device=cuda)
    g = [Fn.gram(X) for _ in range(3)]
    assert torch.equal(g[0], g[1]) and torch.equal(g[0], g[2])
    assert torch.equal(g[0], g[0].t())  # symmetric by construction (mirrored tiles)
    Xb = torch.randn(200, 4096, device=cuda)
    gb = [Fn.gram(Xb) for _ in range(2)]
    assert torch.equal(gb[0], gb[1])
    ref = Xb.double() @ Xb.double().t()
    assert ((gb[0].double() - ref).abs().max() / ref.abs().max()).item() < 1e-5
    with pytest.raises(ValueError, match="128"):
        Fn.coord_select(torch.randn(129, 64, device=cuda), "median")


def test_prep_images(cuda):
    src = torch.randint(0, 256, (50, 32, 32, 3), dtype=torch.uint8)
    idx = torch.randint(0, 50, (2, 7), dtype=torch.int32)
    mean = torch.tensor([0.4914, 0.4822, 0.4465]); inv = 1 / torch.tensor([0.247, 0.243, 0.261])
    for im2col, pad in ((False, 0), (True, 1)):
        a = Fn.prep_images(src.to(cuda), idx.to(cuda), mean.to(cuda), inv.to(cuda), 32, im2col, pad)
        b = Fn.prep_images(src, idx, mean, inv, 32, im2col, pad)
        _close(a, b, rel=1e-2)
    x = torch.randn(4, 1, 28, 28)
    _close(Fn.nchw_to_nhwc(x.to(cuda), 32, True, 0), Fn.nchw_to_nhwc(x, 32, True, 0))
    # the 32-channel stem fast path (CIFAR 3x3x3, MNIST 3x3x1) == the generic kernel (cpad 40)
    for shape, m, s, pad in (((50, 32, 32, 3), mean, inv, 1), ((50, 28, 28, 1), mean[:1], inv[:1], 0)):
        src = torch.randint(0, 256, shape, dtype=torch.uint8)
        args = (src.to(cuda), idx.to(cuda), m.to(cuda), s.to(cuda))
        fast = Fn.prep_images(*args, 32, True, pad)
        generic = Fn.prep_images(*args, 40, True, pad)
        assert torch.equal(fast, generic[..., :32].contiguous())
        _close(fast, Fn.prep_images(src, idx, m, s, 32, True, pad), rel=1e-2)
    # the ImageNet 7x7 / stride-2 stem (147 of 160 channels) on its fast path == the generic (168)
    src = torch.randint(0, 256, (6, 37, 41, 3), dtype=torch.uint8)
    args = (src.to(cuda), idx.to(cuda) % 6, mean.to(cuda), inv.to(cuda))
    fast = Fn.prep_images(*args, 160, 7, 3, 2)
    generic = Fn.prep_images(*args, 168, 7, 3, 2)
    assert torch.equal(fast, generic[..., :160].contiguous())
    _close(fast, Fn.prep_images(src, idx % 6, mean, inv, 160, 7, 3, 2), rel=1e-2)


def test_prep_images_labels(cuda):
    """The batch launch gathers the labels too (one launch per training-step batch)."""
    src = torch.randint(0, 256, (300, 32, 32, 3), dtype=torch.uint8, device=cuda)
    labels = torch.randint(0, 10, (300,), dtype=torch.int32, device=cuda)
    mean = torch.tensor([0.4914, 0.4822, 0.4465], device=cuda)
    inv = 1 / torch.tensor([0.247, 0.243, 0.261], device=cuda)
    idx = torch.randint(0, 300, (3, 70), dtype=torch.int32, device=cuda)
    y = torch.empty(3, 70, dtype=torch.int32, device=cuda)
    a = Fn.prep_images(src, idx, mean, inv, 32, True, 1, labels=labels, labels_out=y)
    assert torch.equal(a, Fn.prep_images(src, idx, mean, inv, 32, True, 1))
    assert torch.equal(y, labels[idx.long()])
    # the ImageNet-stem row kernel (7x7 / stride 2 im2col) gathers them too
    y.zero_()
    a = Fn.prep_images(src, idx, mean, inv, 160, 7, 3, 2, labels=labels, labels_out=y)
    assert torch.equal(a, Fn.prep_images(src, idx, mean, inv, 160, 7, 3, 2))
    assert torch.equal(y, labels[idx.long()])


@pytest.mark.parametrize("geom", [ConvGeom(G=2, N=3, H=8, W=8, C=64, K=96, R=3, S=3, stride=1, pad=1),
                                  ConvGeom(G=1, N=2, H=9, W=7, C=128, K=64, R=3, S=3, stride=2, pad=1)])
def test_conv_dgrad_fused_bn_reduce(cuda, geom, monkeypatch):
    """dgrad epilogue = mask + the preceding BN's backward reduce; bn_backward(part=) then matches
    the unfused three-launch backward. (Autotuner off: the bitwise check needs one tile for both.)"""
    from ddl25spring_amd.ops import autotune
    monkeypatch.setattr(autotune, "ENABLED", False)
    g = geom
    dy = _rand(g.G, g.N, g.P, g.Q, g.K, dev=cuda)
    w = _weights(g, cuda)
    xbn = _rand(g.G, g.N, g.H, g.W, g.C, dev=cuda, scale=2.0) + 0.3
    ymask = _rand(g.G, g.N, g.H, g.W, g.C, dev=cuda)
    mean = torch.randn(g.G, g.C, device=cuda) * 0.2 + 0.3
    rstd = torch.rand(g.G, g.C, device=cuda) + 0.5
    gamma = torch.rand(g.G, g.C, device=cuda) + 0.5
    dxm, part = Fn.conv_dgrad(dy, w, g, mask=ymask, bn=(xbn, mean, rstd))
    plain = Fn.conv_dgrad(dy, w, g, mask=ymask)
    assert torch.equal(dxm, plain)
    d = plain.float().reshape(g.G, -1, g.C)
    xh = (xbn.float().reshape(g.G, -1, g.C) - mean[:, None]) * rstd[:, None]
    _close(part.sum(1)[:, 0], d.sum(1), rel=2e-2)
    _close(part.sum(1)[:, 1], (d * xh).sum(1), rel=2e-2)
    dg1, db1 = torch.zeros(g.G, g.C, device=cuda), torch.zeros(g.G, g.C, device=cuda)
    dg2, db2 = torch.zeros(g.G, g.C, device=cuda), torch.zeros(g.G, g.C, device=cuda)
    # the mask recomputed from the BN input (x * scale + shift > 0) == the stored ReLU output's mask
    sc = torch.randn(g.G, g.C, device=cuda)
    sh = torch.randn(g.G, g.C, device=cuda) * 0.3
    relu_out = (xbn.float() * sc[:, None, None, None] + sh[:, None, None, None]).clamp_min(0).to(torch.bfloat16)
    dxa, pa = Fn.conv_dgrad(dy, w, g, mask=relu_out, bn=(xbn, mean, rstd))
    dxb, pb = Fn.conv_dgrad(dy, w, g, bn=(xbn, mean, rstd), mask_bn=(sc, sh))
    assert (dxa.float() - dxb.float()).abs().max().item() <= 1e-2 * dxa.float().abs().max().item()
    _close(pb.sum(1), pa.sum(1), rel=1e-2)
    fused = Fn.bn_backward(dxm, None, xbn, mean, rstd, gamma, dg1, db1, part=part)
    unfused = Fn.bn_backward(plain, None, xbn, mean, rstd, gamma, dg2, db2)
    _close(fused, unfused, rel=2e-2)
    _close(dg1, dg2, rel=2e-2); _close(db1, db2, rel=2e-2)


SPLIT_GEOMS = [GEOMS[0], GEOMS[1], GEOMS[2], GEOMS[6], GEOMS[7],
               ConvGeom(G=1, N=8, H=4, W=4, C=512, K=512, R=3, S=3, stride=1, pad=1)]  # layer-4, 1 client


@pytest.mark.parametrize("split", [0, 3])
@pytest.mark.parametrize("geom", SPLIT_GEOMS, ids=lambda g: f"{g.C}x{g.K}_{g.H}_{g.R}s{g.stride}p{g.pad}")
def test_conv_split_k(cuda, geom, split):
    """FWD / DGRAD split-K (fp32 partial slices + streaming epilogue) == the direct epilogue: bias,
    relu, BN statistics, residual, mask and the fused BN backward reduce. split 0 = automatic."""
    g = geom
    x = _rand(g.G, g.N, g.H, g.W, g.C, dev=cuda)
    w = _weights(g, cuda)
    bias = torch.randn(g.G, g.K, device=cuda)
    st1, st2 = Fn.stats_buffer(g.G, g.K, cuda), Fn.stats_buffer(g.G, g.K, cuda)
    y1 = Fn.conv_fwd(x, w, g, bias=bias, relu=True, stats=st1, split_k=1)
    y2 = Fn.conv_fwd(x, w, g, bias=bias, relu=True, stats=st2, split_k=split)
    _close(y2, ref.conv_fwd(x.cpu(), w.cpu(), g, bias=bias.cpu(), relu=True))
    _close(y2, y1, rel=1e-2)
    _close(st2.sum(1), st1.sum(1), rel=1e-2)
    dy = _rand(g.G, g.N, g.P, g.Q, g.K, dev=cuda)
    res = _rand(g.G, g.N, g.H, g.W, g.C, dev=cuda)
    mask = _rand(g.G, g.N, g.H, g.W, g.C, dev=cuda)
    dx = Fn.conv_dgrad(dy, w, g, residual=res, mask=mask, split_k=split)
    _close(dx, ref.conv_dgrad(dy.cpu(), w.cpu(), g, residual=res.cpu(), mask=mask.cpu()))
    xbn = _rand(g.G, g.N, g.H, g.W, g.C, dev=cuda) + 0.3
    mean = torch.randn(g.G, g.C, device=cuda) * 0.2
    rstd = torch.rand(g.G, g.C, device=cuda) + 0.5
    dxa, pa = Fn.conv_dgrad(dy, w, g, mask=mask, bn=(xbn, mean, rstd), split_k=1)
    dxb, pb = Fn.conv_dgrad(dy, w, g, mask=mask, bn=(xbn, mean, rstd), split_k=split)
    _close(dxb, dxa, rel=1e-2)
    _close(pb.sum(1), pa.sum(1), rel=2e-2)
    sc = torch.randn(g.G, g.C, device=cuda)
    sh = torch.randn(g.G, g.C, device=cuda) * 0.3
    dxc, pc = Fn.conv_dgrad(dy, w, g, bn=(xbn, mean, rstd), mask_bn=(sc, sh), split_k=1)
    dxd, pd_ = Fn.conv_dgrad(dy, w, g, bn=(xbn, mean, rstd), mask_bn=(sc, sh), split_k=split)
    _close(dxd, dxc, rel=1e-2)
    _close(pd_.sum(1), pc.sum(1), rel=2e-2)


PAIR_GEOMS = [
    ConvGeom(G=1, N=4, H=32, W=32, C=64, K=64, R=3, S=3, stride=1, pad=1),    # layer 1
    ConvGeom(G=2, N=3, H=16, W=16, C=64, K=128, R=3, S=3, stride=2, pad=1),   # stride-2 (phased)
    ConvGeom(G=1, N=5, H=8, W=8, C=256, K=256, R=3, S=3, stride=1, pad=1),    # layer 3, ragged tiles
    ConvGeom(G=2, N=3, H=8, W=8, C=128, K=256, R=1, S=1, stride=2, pad=0),    # projection shortcut
]


@pytest.mark.parametrize("geom", PAIR_GEOMS, ids=lambda g: f"{g.C}x{g.K}_{g.H}_{g.R}s{g.stride}")
def test_conv_pair(cuda, geom):
    """DGRAD + WGRAD in one paired grid == the fp32 references, for every (DGRAD, WGRAD) tile of
    the paired menu the shape admits, with the training epilogue (residual, mask, BN-backward
    reduce) and split-K WGRAD accumulating into a strided view; the tuned entry point agrees."""
    g = geom
    x = _rand(g.G, g.N, g.H, g.W, g.C, dev=cuda)
    w = _weights(g, cuda)
    dy = _rand(g.G, g.N, g.P, g.Q, g.K, dev=cuda)
    res = _rand(g.G, g.N, g.H, g.W, g.C, dev=cuda)
    mask = _rand(g.G, g.N, g.H, g.W, g.C, dev=cuda)
    mean = torch.randn(g.G, g.C, device=cuda) * 0.1
    rstd = torch.rand(g.G, g.C, device=cuda) + 0.5
    dx_ref = ref.conv_dgrad(dy.cpu(), w.cpu(), g, residual=res.cpu(), mask=mask.cpu())
    xh = (x.float() - mean[:, None, None, None]) * rstd[:, None, None, None]
    s0_ref = dx_ref.float().sum((1, 2, 3))
    s1_ref = (dx_ref.float() * xh.cpu()).sum((1, 2, 3))
    dw_ref = torch.zeros(g.G, g.K, g.R, g.S, g.C)
    ref.conv_wgrad(dy.cpu(), x.cpu(), g, dw_ref)
    inner = g.K * g.R * g.S * g.C
    ran = 0
    for bp, bq, bk, ns, halo in Fn.PAIR_DGRAD:
        dcfg = Fn.conv_cfg(bp, bq, bk, ns, halo)
        for wt in Fn.PAIR_WGRAD:
            wcfg = Fn.conv_cfg(*wt)
            for wsp in (1, 3):
                flat = torch.zeros(g.G, inner + 64, device=cuda)
                dw = flat[:, 32:32 + inner].unflatten(1, (g.K, g.R, g.S, g.C))
                try:
                    dx, part = Fn.conv_pair(dy, w, x, g, dw, dcfg, 1, wcfg, wsp, residual=res, mask=mask,
                                            bn=(x, mean, rstd))
                except RuntimeError:
                    continue  # tile not eligible for this shape (or reduction step)
                ran += 1
                _close(dx, dx_ref)
                _close(part[:, :, 0].sum(1), s0_ref, rel=5e-3)
                _close(part[:, :, 1].sum(1), s1_ref, rel=5e-3)
                _close(dw, dw_ref, rel=2e-3)
                assert flat[:, :32].abs().max().item() == 0 and flat[:, 32 + inner:].abs().max().item() == 0
    assert ran > 0
    dw = torch.zeros(g.G, g.K, g.R, g.S, g.C, device=cuda)
    dx, part = Fn.conv_dgrad_wgrad(dy, w, x, g, dw, residual=res, mask=mask, bn=(x, mean, rstd))
    _close(dx, dx_ref)
    _close(dw, dw_ref, rel=2e-3)


FWD_PAIR_GEOMS = [  # (block's last 3x3 conv, its 1x1 / stride-2 shortcut)
    (ConvGeom(G=1, N=4, H=16, W=16, C=128, K=128, R=3, S=3, stride=1, pad=1),
     ConvGeom(G=1, N=4, H=32, W=32, C=64, K=128, R=1, S=1, stride=2, pad=0)),
    (ConvGeom(G=2, N=3, H=4, W=4, C=512, K=512, R=3, S=3, stride=1, pad=1),
     ConvGeom(G=2, N=3, H=8, W=8, C=256, K=512, R=1, S=1, stride=2, pad=0)),
]


@pytest.mark.parametrize("geoms", FWD_PAIR_GEOMS, ids=lambda gs: f"{gs[0].K}_{gs[0].H}")
def test_conv_fwd_pair(cuda, geoms):
    """Two FWD convs in one paired grid (a downsample block's last conv + its shortcut) == the fp32
    references, outputs and BN statistics, for every (A, B) tile of the paired menu the shapes
    admit (A also split-K); the tuned entry point agrees."""
    ga, gb = geoms
    xa, wa = _rand(ga.G, ga.N, ga.H, ga.W, ga.C, dev=cuda), _weights(ga, cuda)
    xb, wb = _rand(gb.G, gb.N, gb.H, gb.W, gb.C, dev=cuda), _weights(gb, cuda)
    ya_ref = ref.conv_fwd(xa.cpu(), wa.cpu(), ga)
    yb_ref = ref.conv_fwd(xb.cpu(), wb.cpu(), gb)

    def stats_ok(st, y):
        _close(st[:, :, 0].sum(1), y.float().sum((1, 2, 3)), rel=5e-3)
        _close(st[:, :, 1].sum(1), y.float().square().sum((1, 2, 3)), rel=5e-3)

    ran = 0
    for ta in Fn.PAIR_FWD_A:
        for tb in Fn.PAIR_FWD_B:
            for asp in (1, 2):
                sa, sb = Fn.stats_buffer(ga.G, ga.K, cuda), Fn.stats_buffer(gb.G, gb.K, cuda)
                try:
                    ya, yb = Fn.conv_fwd_pair(xa, wa, ga, sa, Fn.conv_cfg(*ta), asp, xb, wb, gb, sb,
                                              Fn.conv_cfg(*tb))
                except RuntimeError:
                    continue  # tile not eligible for these shapes
                ran += 1
                _close(ya, ya_ref)
                _close(yb, yb_ref)
                stats_ok(sa.cpu(), ya_ref)
                stats_ok(sb.cpu(), yb_ref)
    assert ran > 0
    sa, sb = Fn.stats_buffer(ga.G, ga.K, cuda), Fn.stats_buffer(gb.G, gb.K, cuda)
    ya, yb = Fn.conv_fwd2(xa, wa, ga, sa, xb, wb, gb, sb)
    _close(ya, ya_ref)
    _close(yb, yb_ref)
    stats_ok(sa.cpu(), ya_ref)
    stats_ok(sb.cpu(), yb_ref)


SUB2_GEOMS = [
    ConvGeom(G=2, N=3, H=16, W=16, C=64, K=128, R=3, S=3, stride=2, pad=1),   # BasicBlock conv1 (phased)
    ConvGeom(G=1, N=2, H=8, W=8, C=128, K=64, R=1, S=1, stride=1, pad=0),     # Bottleneck conv1 (unphased)
    ConvGeom(G=1, N=3, H=7, W=7, C=64, K=64, R=3, S=3, stride=2, pad=1),      # odd size
]


@pytest.mark.parametrize("geom", SUB2_GEOMS, ids=lambda g: f"{g.C}x{g.K}_{g.H}_{g.R}s{g.stride}")
def test_conv_dgrad_residual_sub2(cuda, geom):
    """A compact stride-2 residual (the 1x1 / stride-2 shortcut's input gradient) adds to the (2i, 2j)
    pixels of dx only: single launch, forced split-K (the split epilogue's path), tuned pair."""
    g = geom
    dy = _rand(g.G, g.N, g.P, g.Q, g.K, dev=cuda)
    w = _weights(g, cuda)
    x = _rand(g.G, g.N, g.H, g.W, g.C, dev=cuda)
    res = _rand(g.G, g.N, (g.H + 1) // 2, (g.W + 1) // 2, g.C, dev=cuda)
    mask = _rand(g.G, g.N, g.H, g.W, g.C, dev=cuda)
    full = Fn.expand_sub2(res.cpu(), g.H, g.W)
    dx_ref = ref.conv_dgrad(dy.cpu(), w.cpu(), g, residual=full, mask=mask.cpu())
    _close(Fn.conv_dgrad(dy, w, g, residual=res, mask=mask, residual_sub=2), dx_ref)
    _close(Fn.conv_dgrad(dy, w, g, residual=res, mask=mask, residual_sub=2, split_k=2), dx_ref)
    dw = torch.zeros(g.G, g.K, g.R, g.S, g.C, device=cuda)
    dx = Fn.conv_dgrad_wgrad(dy, w, x, g, dw, residual=res, mask=mask, residual_sub=2)
    _close(dx, dx_ref)
    dw_ref = torch.zeros(g.G, g.K, g.R, g.S, g.C)
    ref.conv_wgrad(dy.cpu(), x.cpu(), g, dw_ref)
    _close(dw, dw_ref, rel=2e-3)
    # the CPU op path agrees with the reference composition
    _close(Fn.conv_dgrad(dy.cpu(), w.cpu(), g, residual=res.cpu(), mask=mask.cpu(), residual_sub=2), dx_ref)


HEAD_CASES = [  # (G, N, H, W, C, Kp, ncls, bias, bn)
    (2, 7, 4, 4, 512, 32, 10, True, True),     # ResNet-18 CIFAR head, fused with the last BN
    (1, 5, 2, 3, 64, 64, 33, False, False),    # plain pool backward, no bias
    (3, 4, 1, 1, 256, 64, 64, True, True),     # 1x1 input, 64 classes (one lane each)
    (1, 40, 7, 7, 2048, 32, 8, True, True),    # ResNet-50-size input (re-read path), 33 samples/block row
]


@pytest.mark.parametrize("case", HEAD_CASES, ids=lambda c: f"C{c[4]}_k{c[6]}_bn{int(c[8])}")
def test_head_train(cuda, case):
    """The fused classifier head (pool -> Linear -> CE -> Linear grads -> pool backward [+ BN mask
    and reduce]) == its fp32 reference."""
    G, N, H, W, C, Kp, ncls, bias, bn = case
    x = _rand(G, N, H, W, C, dev=cuda).relu()
    flat = _rand(G, Kp * C + 64, dev=cuda, scale=0.05)
    w = flat[:, 32:32 + Kp * C].unflatten(1, (Kp, 1, 1, C))       # group-strided, like the store
    b = (torch.randn(G, Kp + 3, device=cuda) * 0.1)[:, :Kp] if bias else None
    labels = torch.randint(0, ncls, (G, N), dtype=torch.int32, device=cuda)
    c = _rand(G, N, H, W, C, dev=cuda)
    mean = torch.randn(G, C, device=cuda) * 0.1
    rstd = torch.rand(G, C, device=cuda) + 0.5
    bnt = (c, mean, rstd) if bn else None
    dw_ref = torch.zeros(G, Kp, 1, 1, C)
    db_ref = torch.zeros(G, Kp) if bias else None
    loss_r, corr_r, dx_r, part_r = Fn.head_train(
        x.cpu(), w.cpu(), None if b is None else b.cpu(), labels.cpu(), ncls, 1.0 / N, dw_ref, db_ref,
        bn=None if bnt is None else tuple(t.cpu() for t in bnt), with_correct=True)
    for _ in range(2):  # the second call accumulates into fresh buffers identically
        gflat = torch.zeros(G, Kp * C + 40, device=cuda)
        dw = gflat[:, 8:8 + Kp * C].unflatten(1, (Kp, 1, 1, C))
        db = torch.zeros(G, Kp, device=cuda) if bias else None
        loss, corr, dx, part = Fn.head_train(x, w, b, labels, ncls, 1.0 / N, dw, db, bn=bnt,
                                             with_correct=True)
        _close(loss, loss_r, rel=1e-3)
        assert torch.equal(corr.cpu(), corr_r), (corr, corr_r)
        _close(dw, dw_ref, rel=2e-3)
        assert gflat[:, :8].abs().max().item() == 0 and gflat[:, 8 + Kp * C:].abs().max().item() == 0
        if bias:
            _close(db, db_ref, rel=2e-3)
        _close(dx, dx_r, rel=1e-2)
        if bn:
            _close(part.sum(1), part_r.sum(1), rel=5e-3)


@pytest.mark.parametrize("G,P,W,gmax", [(3, 1001, 4, 3), (2, 64, 2, 4), (0, 10, 3, 1), (5, 333, 1, 5)])
def test_pack_shards(cuda, G, P, W, gmax):
    """The all-to-all send buffer of the coordinate-sharded aggregators in one pass (aggregate.hip
    pack_shards) == the torch zero / pad / transpose composition."""
    S = -(-P // W)
    rows = torch.randn(G, P + 7)[:, :P]  # a row stride larger than P
    got = Fn.pack_shards(rows.to(cuda), W, S, gmax).cpu()
    want = Fn.pack_shards(rows.contiguous(), W, S, gmax)
    assert torch.equal(got, want)


@pytest.mark.parametrize("K,f,m", [(5, 1, 1), (8, 2, 1), (33, 4, 3), (100, 20, 2), (128, 10, 1)])
def test_krum_select_and_indexed_mean(cuda, K, f, m):
    """Krum scores / selection on the device (aggregate.hip krum_select, a register bitonic sort per
    client) and the winners' mean by index (mean_rows_idx) vs the torch reference."""
    torch.manual_seed(K)
    X = torch.randn(K, 3000)
    X[: f] *= 5.0  # f far-away clients
    g = (X.double() @ X.double().t()).float()
    nb = max(1, K - f - 2)
    sc, sel = Fn.krum_select(g.to(cuda), nb, m)
    sc_ref, sel_ref = Fn.krum_select(g, nb, m)
    assert torch.allclose(sc.cpu(), sc_ref, rtol=1e-5)
    assert sel.cpu().tolist() == sel_ref.tolist()
    out = Fn.mean_rows_idx(X.to(cuda), sel)
    want = Fn.mean_rows_idx(X, sel.cpu())
    assert torch.equal(out.cpu(), want)
