"""Reference-precision (fp32) device path: every fp32 kernel against a float64 PyTorch oracle of
the same op, the whole ResNet-18 training step against torch, and bitwise determinism.

The reference trains in fp32 (lab/tutorial_1a/hfl_complete.py:39-80, stock nn.Conv2d / Linear /
BatchNorm); tolerances here are 1e-5 of the result's max-abs per kernel and 1e-4 per gradient
tensor for the whole network — an exact-fp32 MFMA path (v_mfma_f32_16x16x4_f32) meets them, a
bf16 / TF32-class path would not.
"""
import copy
import hashlib

import pytest
import torch
import torch.nn.functional as F

from ddl25spring_amd.ops import functional as Fn
from ddl25spring_amd.ops import functional_f32 as F32
from ddl25spring_amd.ops.functional import ConvGeom

pytestmark = pytest.mark.gpu


@pytest.fixture(params=["mfma32", "x6", "auto"])
def fmath(request):
    """Both fp32 product engines — the exact fp32 MFMA and the 3-way-split bf16 MFMA (x6) — and
    the default per-layer mix of the two (auto: the tuned plans pick the engine)."""
    old = F32.math()
    F32.set_math(request.param)
    yield request.param
    F32.set_math(old)


def _err(a, b):
    a = a.double().cpu()
    b = b.double().cpu()
    return (a - b).abs().max().item() / (b.abs().max().item() + 1e-30)


def _close(a, b, rel=1e-5):
    e = _err(a, b)
    assert e <= rel, f"relative max err {e:.3g} > {rel:g}"


def _nchw(t):
    return t.permute(0, 3, 1, 2)


def ref_fwd(x, w, g):
    return torch.stack([F.conv2d(_nchw(x[i].double()), w[i].double().permute(0, 3, 1, 2), None, g.stride, g.pad)
                        .permute(0, 2, 3, 1) for i in range(g.G)])


def ref_dgrad(dy, w, g):
    return torch.stack([torch.nn.grad.conv2d_input((g.N, g.C, g.H, g.W), w[i].double().permute(0, 3, 1, 2),
                                                   _nchw(dy[i].double()), g.stride, g.pad).permute(0, 2, 3, 1)
                        for i in range(g.G)])


def ref_wgrad(dy, x, g):
    return torch.stack([torch.nn.grad.conv2d_weight(_nchw(x[i].double()), (g.K, g.C, g.R, g.S), _nchw(dy[i].double()),
                                                    g.stride, g.pad).permute(0, 2, 3, 1) for i in range(g.G)])


GEOMS = [
    ConvGeom(G=2, N=3, H=8, W=8, C=32, K=64, R=3, S=3, stride=1, pad=1),
    ConvGeom(G=1, N=2, H=9, W=9, C=64, K=128, R=3, S=3, stride=2, pad=1),
    ConvGeom(G=3, N=4, H=4, W=4, C=128, K=64, R=1, S=1, stride=2, pad=0),
    ConvGeom(G=2, N=37, H=1, W=1, C=96, K=32, R=1, S=1, stride=1, pad=0),      # Linear
    ConvGeom(G=1, N=2, H=26, W=26, C=32, K=64, R=3, S=3, stride=1, pad=0),
    ConvGeom(G=2, N=4, H=8, W=8, C=256, K=256, R=3, S=3, stride=1, pad=1),
    ConvGeom(G=2, N=3, H=7, W=5, C=64, K=64, R=3, S=3, stride=2, pad=1),      # odd sizes, phases
    ConvGeom(G=1, N=2, H=5, W=6, C=32, K=64, R=1, S=1, stride=2, pad=0),      # 1x1/2: empty phases
    ConvGeom(G=1, N=2, H=9, W=9, C=32, K=32, R=3, S=3, stride=3, pad=1),      # stride 3 (unphased)
    ConvGeom(G=1, N=2, H=16, W=16, C=32, K=64, R=7, S=7, stride=2, pad=3),    # 7x7/2 stem shape
    ConvGeom(G=2, N=5, H=32, W=32, C=64, K=64, R=3, S=3, stride=1, pad=1),    # ResNet layer-1 shape
    ConvGeom(G=1, N=3, H=4, W=4, C=512, K=512, R=3, S=3, stride=1, pad=1),    # layer-4: deep K, split-K
]
IDS = [f"{g.C}x{g.K}_{g.H}x{g.W}_{g.R}s{g.stride}p{g.pad}" for g in GEOMS]


def _weights(geom, dev):
    """Group-strided view into a flat [G, P] buffer, like the flat parameter store."""
    inner = geom.K * geom.R * geom.S * geom.C
    flat = torch.randn(geom.G, inner + 96, device=dev) * 0.1
    return flat[:, 16:16 + inner].unflatten(1, (geom.K, geom.R, geom.S, geom.C))


@pytest.mark.parametrize("geom", GEOMS, ids=IDS)
def test_conv_f32_fwd(cuda, geom, fmath):
    torch.manual_seed(0)
    x = torch.randn(geom.G, geom.N, geom.H, geom.W, geom.C, device=cuda)
    w = _weights(geom, cuda)
    st = F32.SlotStats()
    y = Fn.conv_fwd(x, w, geom, stats=st)
    yr = ref_fwd(x.cpu(), w.cpu(), geom)
    _close(y, yr)
    # per-tile slots: (sum, M2 about the tile's own mean) of st.rows consecutive output rows
    t = st.t.double().cpu()
    yf = yr.reshape(geom.G, -1, geom.K)
    M, rows = yf.shape[1], st.rows
    assert rows > 0 and t.shape[1] == -(-M // rows)
    for i in range(t.shape[1]):
        blk = yf[:, i * rows:(i + 1) * rows]
        _close(t[:, i, 0], blk.sum(1))
        _close(t[:, i, 1], ((blk - blk.mean(1, keepdim=True)) ** 2).sum(1))
    # bias + residual + relu epilogue
    bias = torch.randn(geom.G, geom.K, device=cuda)
    res = torch.randn(geom.G, geom.N, geom.P, geom.Q, geom.K, device=cuda)
    y2 = Fn.conv_fwd(x, w, geom, bias=bias, relu=True, residual=res)
    _close(y2, (yr + bias.cpu().double()[:, None, None, None] + res.cpu().double()).clamp_min(0))
    # operand-side BN: conv(relu(x * scale + shift)), zero padding untouched
    sc = torch.rand(geom.G, geom.C, device=cuda) + 0.5
    sh = torch.randn(geom.G, geom.C, device=cuda) * 0.3
    y3 = Fn.conv_fwd(x, w, geom, in_bn=(sc, sh))
    xa = (x.double() * sc.double()[:, None, None, None] + sh.double()[:, None, None, None]).clamp_min(0)
    _close(y3, ref_fwd(xa.cpu(), w.cpu(), geom))


@pytest.mark.parametrize("geom", GEOMS, ids=IDS)
def test_conv_f32_dgrad(cuda, geom, fmath):
    torch.manual_seed(1)
    dy = torch.randn(geom.G, geom.N, geom.P, geom.Q, geom.K, device=cuda)
    w = _weights(geom, cuda)
    dxr = ref_dgrad(dy.cpu(), w.cpu(), geom)
    _close(Fn.conv_dgrad(dy, w, geom), dxr)
    res = torch.randn(geom.G, geom.N, geom.H, geom.W, geom.C, device=cuda)
    mask = torch.randn(geom.G, geom.N, geom.H, geom.W, geom.C, device=cuda)
    d2 = Fn.conv_dgrad(dy, w, geom, residual=res, mask=mask)
    _close(d2, (dxr + res.cpu().double()) * (mask.cpu() > 0))
    # fused BN-backward reduce with the ReLU mask recomputed from the BN input
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
    xh = (bx.cpu().double() - b(mean)) * b(rstd)
    p = part.double().sum(1).cpu()
    _close(p[:, 0], want.reshape(geom.G, -1, geom.C).sum(1), rel=2e-5)
    _close(p[:, 1], (want * xh).reshape(geom.G, -1, geom.C).sum(1), rel=2e-5)


@pytest.mark.parametrize("stride", [1, 2])
def test_conv_f32_dgrad_compact_residual(cuda, stride, fmath):
    """residual_sub=2: a 1x1/2 shortcut's input gradient added on the (2i, 2j) pixels only (the
    downsample block's first 3x3 conv has stride 2: its DGRAD runs in sub-pixel phases)."""
    geom = ConvGeom(G=2, N=3, H=9, W=8, C=64, K=64, R=3, S=3, stride=stride, pad=1)
    dy = torch.randn(geom.G, geom.N, geom.P, geom.Q, geom.K, device=cuda)
    w = _weights(geom, cuda)
    rc = torch.randn(geom.G, geom.N, 5, 4, geom.C, device=cuda)
    d = Fn.conv_dgrad(dy, w, geom, residual=rc, residual_sub=2)
    _close(d, ref_dgrad(dy.cpu(), w.cpu(), geom) + Fn.expand_sub2(rc, 9, 8).cpu().double())


@pytest.mark.parametrize("geom", GEOMS, ids=IDS)
def test_conv_f32_wgrad(cuda, geom, fmath):
    torch.manual_seed(2)
    x = torch.randn(geom.G, geom.N, geom.H, geom.W, geom.C, device=cuda)
    dy = torch.randn(geom.G, geom.N, geom.P, geom.Q, geom.K, device=cuda)
    inner = geom.K * geom.R * geom.S * geom.C
    flat = torch.zeros(geom.G, inner + 64, device=cuda)
    dw = flat[:, 32:32 + inner].unflatten(1, (geom.K, geom.R, geom.S, geom.C))
    Fn.conv_wgrad(dy, x, geom, dw, accumulate=True)
    dwr = ref_wgrad(dy.cpu(), x.cpu(), geom)
    _close(dw, dwr)
    assert flat[:, :32].abs().max().item() == 0 and flat[:, 32 + inner:].abs().max().item() == 0
    # scaled accumulate (direct SGD: w += -lr * dW) and the operand-side BN of x
    w0 = torch.randn_like(dw)
    wt = w0.clone()
    F32.conv_wgrad(dy, x, geom, wt, accumulate=True, gscale=-0.05)
    _close(wt, w0.cpu().double() - 0.05 * dwr, rel=1e-5)
    sc = torch.rand(geom.G, geom.C, device=cuda) + 0.5
    sh = torch.randn(geom.G, geom.C, device=cuda) * 0.3
    dw2 = torch.zeros_like(dw)
    Fn.conv_wgrad(dy, x, geom, dw2, accumulate=True, in_bn=(sc, sh))
    xa = (x.double() * sc.double()[:, None, None, None] + sh.double()[:, None, None, None]).clamp_min(0)
    _close(dw2, ref_wgrad(dy.cpu(), xa.cpu(), geom))


def test_conv_f32_tiles_and_splits_deterministic(cuda, fmath):
    """Every tile config x split-K count gives the same math; each is bitwise reproducible."""
    geom = ConvGeom(G=2, N=3, H=8, W=8, C=128, K=128, R=3, S=3, stride=2, pad=1)
    torch.manual_seed(3)
    x = torch.randn(geom.G, geom.N, geom.H, geom.W, geom.C, device=cuda)
    w = _weights(geom, cuda)
    dy = torch.randn(geom.G, geom.N, geom.P, geom.Q, geom.K, device=cuda)
    refs = (ref_fwd(x.cpu(), w.cpu(), geom), ref_dgrad(dy.cpu(), w.cpu(), geom), ref_wgrad(dy.cpu(), x.cpu(), geom))
    try:
        for bp in (64, 128):
            for bq in (64, 128):
                for split in (1, 2, 3, 5):
                    for mode in (F32.F_FWD, F32.F_DGRAD, F32.F_WGRAD):
                        F32.set_plan(mode, geom, bp, bq, split)
                    outs = []
                    for _ in range(2):
                        dw = torch.zeros(geom.G, geom.K, geom.R, geom.S, geom.C, device=cuda)
                        Fn.conv_wgrad(dy, x, geom, dw)
                        outs.append((Fn.conv_fwd(x, w, geom), Fn.conv_dgrad(dy, w, geom), dw))
                    for got, r in zip(outs[0], refs):
                        _close(got, r)
                    for a, b in zip(*outs):
                        assert torch.equal(a, b), (bp, bq, split)
    finally:
        F32._OVERRIDE.clear()
        F32._PLANS.clear()


# ------------------------------------------------------------------------------ BN / head passes
def _bn_ref(c, gamma, beta, eps=1e-5):
    """float64 training-mode BN over [G, M, C] -> y, mean, var."""
    mean = c.mean(1, keepdim=True)
    var = c.var(1, unbiased=False, keepdim=True)
    return (c - mean) / torch.sqrt(var + eps) * gamma[:, None] + beta[:, None], mean[:, 0], var[:, 0]


def test_bn_f32_forward_backward(cuda):
    torch.manual_seed(4)
    G, M, C = 2, 777, 64
    c = torch.randn(G, M, C, device=cuda) * 2 + 0.5
    gamma = torch.rand(G, C, device=cuda) + 0.5
    beta = torch.randn(G, C, device=cuda) * 0.1
    rm, rv = torch.zeros(G, C, device=cuda), torch.ones(G, C, device=cuda)
    stats = Fn.bn_stats(c)
    sc, sh, mu, rs = Fn.bn_finalize(stats, gamma, beta, rm, rv, M)
    c64 = c.double().cpu().requires_grad_(True)
    y64, mean64, var64 = _bn_ref(c64, gamma.double().cpu(), beta.double().cpu())
    _close(mu, mean64)
    _close(rs, 1 / torch.sqrt(var64 + 1e-5))
    _close(rm, 0.1 * mean64)
    _close(rv, 0.9 + 0.1 * var64 * M / (M - 1))
    r = torch.randn_like(c)
    y = Fn.bn_apply(c, sc, sh, r=r, act=1)
    _close(y, (y64 + r.cpu().double()).clamp_min(0).detach())
    # backward through the ReLU mask of y, d(gamma) / d(beta) accumulated into the given views
    dy = torch.randn_like(c)
    dgamma, dbeta = torch.full((G, C), 0.25, device=cuda), torch.full((G, C), -0.5, device=cuda)
    dx = Fn.bn_backward(dy, y, c, mu, rs, gamma, dgamma, dbeta)
    m = (y64 + r.cpu().double()) > 0
    y64.backward(dy.cpu().double() * m)
    _close(dx, c64.grad)
    want_db = (dy.cpu().double() * m).sum(1)
    _close(dbeta, want_db - 0.5)
    xh = (c64.detach() - mean64[:, None]) / torch.sqrt(var64[:, None] + 1e-5)
    _close(dgamma, (dy.cpu().double() * m * xh).sum(1) + 0.25)


def test_bn_f32_backward2_and_reduce_part(cuda):
    torch.manual_seed(5)
    G, M, C = 3, 300, 128
    dy = torch.randn(G, M, C, device=cuda)
    bns, refs = [], []
    for _ in range(2):
        c = torch.randn(G, M, C, device=cuda)
        mean, var = c.mean(1), c.var(1, unbiased=False)
        rstd = 1 / torch.sqrt(var + 1e-5)
        gamma = torch.rand(G, C, device=cuda) + 0.5
        dg, db = torch.zeros(G, C, device=cuda), torch.zeros(G, C, device=cuda)
        part = Fn.bn_bwd_reduce_part(dy, None, c, mean, rstd)
        bns.append((c, mean, rstd, gamma, dg, db, part))
        c64 = c.double().cpu().requires_grad_(True)
        y64, _, _ = _bn_ref(c64, gamma.double().cpu(), torch.zeros(G, C, dtype=torch.float64))
        y64.backward(dy.double().cpu())
        refs.append(c64.grad)
    dxa, dxb = Fn.bn_backward2(dy, bns[0], bns[1])
    _close(dxa, refs[0], rel=2e-5)
    _close(dxb, refs[1], rel=2e-5)


@pytest.mark.parametrize("G,M,C", [(3, 300, 128), (8, 102400, 64), (1, 1600, 512)])
def test_bn_f32_one_launch_fold_equals_two_launch(cuda, monkeypatch, G, M, C):
    """bnf_fold_one_kernel (last-arriving block folds the level-1 partials) is bit for bit the two-launch
    fold (bnf_fold_part + bnf_fold_fin), for one BN and for two sharing dy; its arrival counters are
    back at zero after every launch (the next call would otherwise mis-detect its last block)."""
    from ddl25spring_amd.ops import functional_f32 as F32
    torch.manual_seed(9)
    dy = torch.randn(G, M, C, device=cuda)
    bns = []
    for _ in range(2):
        c = torch.randn(G, M, C, device=cuda)
        mean, var = c.mean(1), c.var(1, unbiased=False)
        part = Fn.bn_bwd_reduce_part(dy, None, c, mean, 1 / torch.sqrt(var + 1e-5))
        bns.append((c, mean, 1 / torch.sqrt(var + 1e-5), torch.rand(G, C, device=cuda) + 0.5, part))

    def run():
        outs = []
        for c, mean, rstd, gamma, part in bns:  # one BN
            dg, db = torch.zeros(G, C, device=cuda), torch.zeros(G, C, device=cuda)
            coef = F32.bn_backward_coef(dy, c, mean, rstd, gamma, dg, db, part=part)
            outs += [coef, dg, db]
        two = [(c, mean, rstd, gamma, torch.zeros(G, C, device=cuda), torch.zeros(G, C, device=cuda), part)
               for c, mean, rstd, gamma, part in bns]
        outs += list(Fn.bn_backward2(dy, two[0], two[1])) + [t[4] for t in two] + [t[5] for t in two]
        torch.cuda.synchronize()
        return outs

    monkeypatch.setattr(F32, "FOLD1L", [True])
    one = run()
    F32.ensure_workspace(cuda)
    assert int(F32._TICKETS[F32._dev_key(cuda)].abs().sum()) == 0
    monkeypatch.setattr(F32, "FOLD1L", [False])
    two = run()
    for a, b in zip(one, two):
        assert torch.equal(a, b)


def test_head_f32_matches_torch(cuda):
    """pool -> FC -> softmax CE -> FC grads -> pool backward masked by the block's ReLU + BN reduce."""
    torch.manual_seed(6)
    G, N, H, W, C, K = 2, 37, 4, 4, 512, 10
    c = torch.randn(G, N, H, W, C, device=cuda)
    x = torch.relu(c * 0.7 + 0.1)
    mean, rstd = torch.randn(G, C, device=cuda) * 0.1, torch.rand(G, C, device=cuda) + 0.5
    wflat = torch.randn(G, 32 * C + 64, device=cuda) * 0.05
    w = wflat[:, :32 * C].unflatten(1, (32, 1, 1, C))
    b = torch.randn(G, 32, device=cuda) * 0.1
    dw, db = torch.zeros(G, 32, 1, 1, C, device=cuda), torch.zeros(G, 32, device=cuda)
    lab = torch.randint(0, K, (G, N), device=cuda, dtype=torch.int32)
    loss, correct, dx, part = Fn.head_train(x, w, b, lab, K, 1.0 / N, dw, db, bn=(c, mean, rstd), with_correct=True)
    x64 = x.double().cpu().requires_grad_(True)
    w64 = w.double().cpu().reshape(G, 32, C)[:, :K].requires_grad_(True)
    b64 = b.double().cpu()[:, :K].requires_grad_(True)
    z = torch.einsum("gnc,gkc->gnk", x64.mean((2, 3)), w64) + b64[:, None]
    lr = torch.stack([F.cross_entropy(z[g], lab[g].long().cpu()) for g in range(G)])
    lr.sum().backward()
    _close(loss, lr.detach())
    assert correct.cpu().tolist() == [(z[g].argmax(-1) == lab[g].long().cpu()).sum().item() for g in range(G)]
    _close(dw.reshape(G, 32, C)[:, :K], w64.grad)
    _close(db[:, :K], b64.grad)
    dxr = x64.grad * (x64.detach() > 0)
    _close(dx, dxr)
    xh = (c.double().cpu() - mean.double().cpu()[:, None, None, None]) * rstd.double().cpu()[:, None, None, None]
    p = part.double().sum(1).cpu()
    _close(p[:, 0], dxr.reshape(G, -1, C).sum(1), rel=2e-5)
    _close(p[:, 1], (dxr * xh).reshape(G, -1, C).sum(1), rel=2e-5)


# ------------------------------------------------------------------------------ whole network
def _resnet_pair(cuda, G, seed=0):
    from ddl25spring_amd.models import convert, resnet18_cifar
    from ddl25spring_amd.models.torch_ref import torch_resnet18_cifar
    torch.manual_seed(seed)
    tm = torch_resnet18_cifar(10)
    net = resnet18_cifar(10, groups=G, precision="fp32").to(cuda)
    mapping = convert.resnet_mapping(net)
    convert.import_torch(net, tm, mapping)
    return tm, net, mapping, convert


def test_resnet18_fp32_step_matches_torch(cuda, fmath):
    """One native fp32 ResNet-18 training step (all the fused kernels, fused head) vs torch autograd
    in float64: loss and every parameter gradient within 1e-4 (max-abs relative); also reports
    stock torch fp32 on the GPU for scale."""
    tm, net, mapping, convert = _resnet_pair(cuda, G=2)
    torch.manual_seed(1)
    x = torch.randn(16, 3, 32, 32)
    y = torch.randint(0, 10, (16,))
    net.store.zero_grad()
    xin = net.prepare_input(x.to(cuda))
    assert xin.dtype == torch.float32
    loss, _ = net.train_step(torch.cat([xin, xin]), torch.stack([y, y]).to(cuda, torch.int32))
    t64 = tm.double()
    lt = F.cross_entropy(t64(x.double()), y)
    lt.backward()
    assert abs(loss[0].item() - lt.item()) <= 1e-5 * abs(lt.item())
    assert loss[0].item() == loss[1].item()
    for grp in (0, 1):
        g = convert.export_torch(net, t64, mapping, group=grp, grads=True)
        for name, p in t64.named_parameters():
            e = _err(g[name], p.grad)
            assert e <= 1e-4, (grp, name, e)


def _hash(t):
    return hashlib.sha256(t.detach().cpu().numpy().tobytes()).hexdigest()


def test_fedavg_fp32_deterministic(cuda, fmath):
    """Two fresh FedAvg runs (ResNet-18, fp32, 2 clients, graph-replayed rounds) and an eager run
    produce bitwise-identical server weights: no atomics anywhere in the fp32 step."""
    from ddl25spring_amd.data.images import DeviceImageDataset, synthetic_images
    from ddl25spring_amd.data.split import split
    from ddl25spring_amd.fl.algorithms import FedAvg
    from ddl25spring_amd.models import resnet18_cifar
    train = synthetic_images("cifar10", 400, seed=0)

    def run(graph):
        ds = DeviceImageDataset(train, cuda)
        fl = FedAvg(lambda groups: resnet18_cifar(10, groups=groups, precision="fp32"), ds,
                    split(2, True, 10, labels=train.labels), lr=0.01, batch_size=50, local_epochs=1,
                    client_fraction=1.0, seed=10, use_graph=graph, eval_every=0)
        for _ in range(2):
            fl.round()
        torch.cuda.synchronize()
        return _hash(fl.w_global), fl.w_global.clone()

    h1, w1 = run(True)
    h2, _ = run(True)
    h3, w3 = run(False)
    assert h1 == h2, "graph-replayed fp32 rounds differ run to run"
    assert h1 == h3, f"graph vs eager differ: max {(w1 - w3).abs().max().item()}"


# ------------------------------------------------------------------------------ exactness of the engine
def _fedavg(cuda, model, kind, n, clients, batch, **kw):
    from ddl25spring_amd.data.images import DeviceImageDataset, synthetic_images
    from ddl25spring_amd.data.split import split
    from ddl25spring_amd.fl.algorithms import FedAvg
    from ddl25spring_amd.models import mnist_cnn, resnet18_cifar
    from ddl25spring_amd.runtime.dist import DistContext
    arr = synthetic_images(kind, n, seed=0)
    fn = {"resnet18": resnet18_cifar, "mnist_cnn": mnist_cnn}[model]
    return FedAvg(lambda groups: fn(groups=groups, precision="fp32"), DeviceImageDataset(arr, cuda),
                  split(clients, True, 3, labels=arr.labels), lr=0.05, batch_size=batch, client_fraction=1.0,
                  seed=3, ctx=DistContext(device=cuda), eval_every=0, **kw)


@pytest.mark.parametrize("model,kind,batch", [("mnist_cnn", "mnist", 60), ("resnet18", "cifar10", 50)])
def test_fp32_graph_replay_equals_eager_exactly(cuda, model, kind, batch):
    """fp32: graph-replayed rounds == eager rounds bit for bit (MnistCnn includes dropout, whose
    Philox counter advances on the device; batch 60 leaves a short last step in the graph)."""
    ws = []
    for graph in (True, False):
        fa = _fedavg(cuda, model, kind, 400, 2, batch, use_graph=graph)
        for _ in range(2):
            fa.round()
        ws.append(fa.w_global.clone())
    assert torch.equal(ws[0], ws[1]), (ws[0] - ws[1]).abs().max().item()


@pytest.mark.parametrize("model,kind", [("mnist_cnn", "mnist"), ("resnet18", "cifar10")])
def test_fp32_direct_sgd_equals_gradient_sgd_exactly(cuda, model, kind, monkeypatch):
    """Direct SGD (WGRAD adds -lr * dW into the master weights) == zeroed grads + fused SGD step:
    fl(p + fl(-lr * dW)) == fl(p - fl(lr * dW)), so in fp32 the two are bitwise equal."""
    import ddl25spring_amd.fl.local as L
    ws = []
    for direct in (False, True):
        monkeypatch.setattr(L, "DIRECT_SGD", direct)
        fa = _fedavg(cuda, model, kind, 200, 2, 50, use_graph=True)
        fa.round()
        assert fa.trainer.direct == direct
        st = fa.net.store
        assert st.shadow is st.data and st.shadow16 is None  # fp32: the kernels read the master
        ws.append(fa.w_global.clone())
    assert torch.equal(ws[0], ws[1]), (ws[0] - ws[1]).abs().max().item()


def test_fp32_unsynchronised_rounds_equal_exactly(cuda):
    """bench.py's timed mode (rounds enqueued back to back, no host sync) == synchronised rounds."""
    ws = []
    for sync in (True, False):
        fa = _fedavg(cuda, "resnet18", "cifar10", 400, 4, 50)
        fa.round()
        fa.sync_rounds = sync
        for _ in range(2):
            _, s = fa.round()
            assert s == 400
        torch.cuda.synchronize()
        ws.append(fa.w_global.clone())
    assert torch.equal(ws[0], ws[1])


def test_fp32_mnist_cnn_step_matches_torch(cuda, fmath):
    """The reference's own model (hfl_complete.py:39-64) in fp32 on the device vs torch float64:
    conv+bias+ReLU, maxpool, Linear, log_softmax/NLL — dropout disabled for the comparison."""
    from ddl25spring_amd.models import convert, mnist_cnn
    from ddl25spring_amd.models.torch_ref import TorchMnistCnn
    from ddl25spring_amd.models.zoo import mnist_cnn_mapping
    torch.manual_seed(3)
    tm = TorchMnistCnn()
    net = mnist_cnn(precision="fp32").to(cuda)
    convert.import_torch(net, tm, mnist_cnn_mapping())
    for layer in net.layers:
        if hasattr(layer, "p"):
            layer.p = 0.0
    tm = tm.double().eval()
    x = torch.randn(12, 1, 28, 28)
    y = torch.randint(0, 10, (12,))
    net.store.zero_grad()
    loss, _ = net.train_step(net.prepare_input(x.to(cuda)), y[None].to(cuda, torch.int32))
    lt = F.nll_loss(tm(x.double()), y)
    lt.backward()
    assert abs(loss[0].item() - lt.item()) <= 1e-5 * abs(lt.item())
    g = convert.export_torch(net, tm, mnist_cnn_mapping(), grads=True)
    for name, p in tm.named_parameters():
        assert _err(g[name], p.grad) <= 1e-4, name


def test_resnet50_fp32_step_as_accurate_as_torch_fp32(cuda):
    """BASELINE config 3's model at the reference's precision: one native fp32 ResNet-50 training
    step (bottleneck blocks, 7x7 im2col stem, max pool, 1x1 convs up to 2048 channels, C = 2048
    BN passes; default engine mix) vs torch autograd in float64 on a small ImageNet-shaped batch.

    A 50-layer net whose last BatchNorms see 4 x 4 x 4 values per channel amplifies fp32 rounding
    (ReLU masks flip near zero), so float64 agreement to 1e-4 is out of reach for ANY fp32
    implementation: stock torch fp32 itself lands ~1-2 % (norm-relative) away on some gradients.
    The check is therefore relative to that reference: every parameter gradient of the native
    step is within 3x (+1e-3) of stock torch fp32's own distance from float64, and on aggregate
    (median over parameters) no farther than 2x (+1e-4) of it."""
    from ddl25spring_amd.models import convert, resnet50_imagenet
    from ddl25spring_amd.models.torch_ref import torch_resnet50_imagenet

    def nerr(a, b):
        a, b = a.double().cpu(), b.double().cpu()
        return ((a - b).norm() / (b.norm() + 1e-30)).item()
    torch.manual_seed(0)
    tm = torch_resnet50_imagenet(1000)
    t32 = copy.deepcopy(tm)
    net = resnet50_imagenet(1000, groups=1, precision="fp32").to(cuda)
    mapping = convert.resnet_mapping(net)
    convert.import_torch(net, tm, mapping)
    torch.manual_seed(1)
    x = torch.randn(4, 3, 128, 128)
    y = torch.randint(0, 1000, (4,))
    net.store.zero_grad()
    xin = net.prepare_input(x.to(cuda))
    assert xin.dtype == torch.float32
    loss, _ = net.train_step(xin, y.view(1, -1).to(cuda, torch.int32))
    t64 = tm.double()
    lt = F.cross_entropy(t64(x.double()), y)
    lt.backward()
    F.cross_entropy(t32(x), y).backward()
    assert abs(loss[0].item() - lt.item()) <= 1e-5 * abs(lt.item())
    g = convert.export_torch(net, t64, mapping, group=0, grads=True)
    ours, ref32 = [], []
    for (name, p), p32 in zip(t64.named_parameters(), t32.parameters()):
        ours.append((name, nerr(g[name], p.grad)))
        ref32.append(nerr(p32.grad, p.grad))
    # floor 1e-3: torch's own CPU fp32 error moves with the host's SIMD width and thread count; a
    # real defect (a wrong mask, index or statistic) shows up as >= 1e-2 on these gradients
    bad = [(n, round(e, 6), round(r, 6)) for (n, e), r in zip(ours, ref32) if e > 3 * r + 1e-3]
    assert not bad, bad
    med = sorted(e for _, e in ours)[len(ours) // 2]
    med32 = sorted(ref32)[len(ref32) // 2]
    assert med <= 2 * med32 + 1e-4, (med, med32)


def test_fp32_resnet18_128_step_chunk_graph_equals_eager(cuda):
    """The round-graph chunk size actually shipped (fl/local.py GRAPH_MAX_STEPS = 128): one client,
    ResNet-18, 16-sample batches over 2,072 samples = 129 full steps + a short one, so a round is a
    128-step chunk graph, then a 1-step chunk with the tail -- bit for bit the eager round."""
    import ddl25spring_amd.fl.local as L
    assert L.GRAPH_MAX_STEPS == 128
    ws = []
    for graph in (True, False):
        fa = _fedavg(cuda, "resnet18", "cifar10", 2072, 1, 16, use_graph=graph)
        fa.round()
        ws.append(fa.w_global.clone())
    assert torch.equal(ws[0], ws[1]), (ws[0] - ws[1]).abs().max().item()
