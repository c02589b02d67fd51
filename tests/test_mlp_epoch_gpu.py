"""The one-launch MLP epoch kernel (csrc/kernels/mlp_epoch.hip) against the float64 torch reference
epoch (ops/mlp_epoch.reference_epoch, the SAME Philox dropout masks): parameters, Adam moments,
loss / accuracy statistics and the device step counter after several epochs, with partial last
mini-batches and mini-batches wider than one wave; plus VFLNetwork routing onto it."""
import pytest
import torch

from ddl25spring_amd.models import tabular as T
from ddl25spring_amd.ops import mlp_epoch as ME
from ddl25spring_amd.optim import FlatAdamW

pytestmark = pytest.mark.gpu


def _setup(cuda, feats, drop, n, seed=0):
    torch.manual_seed(seed)
    bottoms = [T.BottomModel(f, 2 * f) for f in feats]
    top = T.TopModel(bottoms, 2)
    for m in [*bottoms, top]:
        m.dropout.p = drop
    g = torch.Generator().manual_seed(seed + 1)
    xs = [torch.randn(n, f, generator=g) for f in feats]
    y = torch.nn.functional.one_hot(torch.randint(0, 2, (n,), generator=g), 2).float()
    return bottoms, top, xs, y


@pytest.mark.parametrize("lr", [0.0, 1e-3])
@pytest.mark.parametrize("feats,drop,n,B", [((15, 15), 0.1, 821, 64), ((7, 13, 10), 0.25, 250, 48),
                                            ((15, 15), 0.3, 300, 40), ((15, 15), 0.0, 130, 64)])
def test_kernel_matches_reference(cuda, feats, drop, n, B, lr):
    """lr = 0: the parameters stay put, so every mini-batch's gradient (g = the last one, m / v =
    the moment sums of all of them) is pinned tightly against float64. lr = 1e-3: the trained run;
    Adam turns fp32-vs-fp64 noise on near-zero gradients into +-lr steps, so the parameters are
    pinned to a few lr and the losses to 1e-3."""
    ME.abi_check()
    bottoms, top, xs, y = _setup(cuda, feats, drop, n)
    # CPU copy of the initial state for the reference
    params = [*[p for b in bottoms for p in b.parameters()], *top.parameters()]
    init = [p.detach().clone() for p in params]
    for m in [*bottoms, top]:
        m.to(cuda)
    opt = FlatAdamW([*[p for b in bottoms for p in b.parameters()], *top.parameters()], lr=lr)
    eng = ME.MlpEpoch(ME.splitnn_graph(bottoms, top), opt, B, seed=1234)
    xg, yg = [x.to(cuda) for x in xs], y.to(cuda)
    epochs = 3
    stats = torch.zeros(epochs, 2, device=cuda)
    for e in range(epochs):
        eng.run(xg, yg, stats[e])
    torch.cuda.synchronize()
    steps = epochs * -(-n // B)
    assert int(opt.t_dev.item()) == steps and opt.t == steps
    # reference: same graph over CPU parameters with the same offsets
    flat = {k: torch.zeros_like(getattr(opt, a), device="cpu", dtype=torch.float64)
            for k, a in (("p", "data"), ("g", "grad"), ("m", "m"), ("v", "v"))}
    offsets = {}
    cpu_params = []
    for p, off, p0 in zip(opt.params, opt.offsets, init):
        flat["p"][off:off + p0.numel()] = p0.reshape(-1).double()
        q = torch.nn.Parameter(p0.clone())
        offsets[id(q)] = off
        cpu_params.append(q)
    # rebuild the graph over the CPU parameters (same structure, same order)
    mp = dict(zip([id(p) for p in opt.params], cpu_params))
    g = ME.splitnn_graph(bottoms, top)
    for L in g.layers:
        L.weight, L.bias = mp[id(L.weight)], mp[id(L.bias)]
    ref_stats = []
    for e in range(epochs):
        ls, cor = ME.reference_epoch(g, flat, offsets, xs, y, B, 1234, e * -(-n // B), opt.lr, opt.betas, opt.eps,
                                     opt.weight_decay, dtype=torch.float64)
        ref_stats.append((ls, cor))
    rel = lambda a, b: ((a.double().cpu() - b).abs().max() / b.abs().max()).item()  # noqa: E731
    st = stats.cpu()
    if lr == 0.0:
        assert torch.equal(opt.data.double().cpu(), flat["p"])
        assert rel(opt.grad, flat["g"]) < 2e-5
        assert rel(opt.m, flat["m"]) < 2e-5 and rel(opt.v, flat["v"]) < 5e-5
        for e, (ls, cor) in enumerate(ref_stats):
            assert abs(st[e, 0].item() - ls) < 1e-5 * max(1.0, abs(ls))
            assert abs(st[e, 1].item() - cor) <= 1  # an argmax tie within rounding may flip
    else:
        d = (opt.data.double().cpu() - flat["p"]).abs()
        assert d.max() < 6 * lr
        assert (d > 0.5 * lr).double().mean() < 0.02  # fewer than 2% are half a step apart
        for e, (ls, cor) in enumerate(ref_stats):
            assert abs(st[e, 0].item() - ls) < 1e-3 * max(1.0, abs(ls))


def test_oversized_batch_is_refused(cuda):
    """A mini-batch whose activations exceed the LDS arena is refused (VFLNetwork then keeps the
    module path)."""
    bottoms, top, xs, y = _setup(cuda, (15, 15), 0.1, 300)
    for m in [*bottoms, top]:
        m.to(cuda)
    opt = FlatAdamW([*[p for b in bottoms for p in b.parameters()], *top.parameters()])
    with pytest.raises(ValueError):
        ME.MlpEpoch(ME.splitnn_graph(bottoms, top), opt, 128)


def test_vfl_network_routes_to_fused_epoch(cuda):
    bottoms, top, xs, y = _setup(cuda, (15, 15), 0.1, 300)
    net = T.VFLNetwork(bottoms, 2)
    net.top_model = top
    net.to(cuda)
    net.optimizer = FlatAdamW(net.parameters())
    eng = net.fused_epoch_engine(64)
    assert eng is not None
    import pandas as pd
    cols = [[f"a{i}" for i in range(15)], [f"b{i}" for i in range(15)]]
    X = pd.DataFrame(torch.cat(xs, 1).numpy(), columns=cols[0] + cols[1])
    Y = pd.DataFrame(y.numpy(), columns=["n", "p"])
    hist = net.train_with_settings(8, 64, 2, cols, X, Y)
    assert len(hist) == 8 and hist[-1][0] < hist[0][0]
    assert 0.0 <= hist[-1][1] <= 1.0
    assert int(net.optimizer.t_dev.item()) == 8 * 5


def test_fused_epoch_golden_party_scaling(cuda):
    """Device golden run on the one-launch epoch engine: lab/homework-2.ipynb:306 (cell 4) setup --
    4 parties on the balanced split of the 30 encoded heart columns, 300 epochs, B=64, seed 42 --
    with the reference's quirks fixed (bottoms optimised, zero_grad per mini-batch: the
    configuration the fused engine serves). Published 84.31 % (quirks on); the fixed net must land
    within 5 pp of it or above. Data: tests/data/heart_vfl.npz (the reference heart.csv after the
    D3 recipe; the reference tree is not on the GPU box)."""
    import numpy as np
    import pandas as pd
    from pathlib import Path
    from ddl25spring_amd.data import heart as H
    z = np.load(Path(__file__).parent / "data" / "heart_vfl.npz", allow_pickle=False)
    X = pd.DataFrame(z["x"], columns=[str(c) for c in z["x_cols"]])
    Y = pd.DataFrame(z["y"], columns=[str(c) for c in z["y_cols"]])
    parts = H.partition_balanced(list(X.columns), 4)
    Xtr, Xte = H.row_split(X)
    Ytr, Yte = H.row_split(Y)
    torch.manual_seed(42)
    bottoms = [T.BottomModel(len(p), 2 * len(p)).to(cuda) for p in parts]
    net = T.VFLNetwork(bottoms, 2).to(cuda)
    net.optimizer = FlatAdamW(net.parameters())
    assert net.fused_epoch_engine(64) is not None
    hist = net.train_with_settings(300, 64, 4, parts, Xtr, Ytr)
    assert int(net.optimizer.t_dev.item()) == 300 * -(-len(Ytr) // 64)  # every step ran in the kernel
    acc = float(net.test(Xte, Yte)[0])
    assert hist[-1][0] < hist[0][0]
    assert acc >= 0.8431 - 0.05, acc
