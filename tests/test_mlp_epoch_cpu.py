"""The one-launch MLP epoch (ops/mlp_epoch.py) on the CPU: its torch reference epoch against the
module path (VFLNetwork mini-batch training with FlatAdamW, dropout off so both see the same
network), the Philox dropout masks, and the graph checks."""
import numpy as np
import pytest
import torch

from ddl25spring_amd.models import tabular as T
from ddl25spring_amd.ops import mlp_epoch as ME
from ddl25spring_amd.optim import FlatAdamW


def _net(feats=(15, 15), drop=0.0, seed=0):
    torch.manual_seed(seed)
    bottoms = [T.BottomModel(f, 2 * f) for f in feats]
    net = T.VFLNetwork(bottoms, 2)
    for m in [*bottoms, net.top_model]:
        m.dropout.p = drop
    return net


def _data(n=150, feats=(15, 15), seed=1):
    g = torch.Generator().manual_seed(seed)
    xs = [torch.randn(n, f, generator=g) for f in feats]
    lab = torch.randint(0, 2, (n,), generator=g)
    y = torch.nn.functional.one_hot(lab, 2).float()
    return xs, y


def test_reference_epoch_matches_module_path():
    xs, y = _data()
    B, epochs = 32, 2
    a, b = _net(), _net()
    for p, q in zip(a.parameters(), b.parameters()):
        assert torch.equal(p, q)
    # module path: zero_grad / forward / CE / backward / AdamW per mini-batch
    oa = FlatAdamW(a.parameters())
    crit = T.SoftCrossEntropy()
    losses = []
    for _ in range(epochs):
        tot = 0.0
        for r0 in range(0, len(y), B):
            oa.zero_grad()
            loss = crit(a([x[r0:r0 + B] for x in xs]), y[r0:r0 + B])
            loss.backward()
            oa.step()
            tot += float(loss.detach())
        losses.append(tot)
    # the fused engine's CPU path (reference_epoch)
    ob = FlatAdamW(b.parameters())
    eng = ME.MlpEpoch(ME.splitnn_graph(list(b.bottom_models), b.top_model), ob, B, seed=7)
    got = []
    for _ in range(epochs):
        st = torch.zeros(2)
        eng.run(xs, y, st)
        got.append(float(st[0]))
    assert ob.t == oa.t == epochs * -(-len(y) // B)
    np.testing.assert_allclose(got, losses, rtol=1e-5)
    torch.testing.assert_close(ob.data, oa.data, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(ob.m, oa.m, rtol=1e-4, atol=1e-7)


def test_keep_mask_rate_and_independence():
    m1 = ME.keep_mask(123, 5, 2, 64, 60, 0, 60, 0.1)
    assert m1.shape == (64, 60)
    assert abs(m1.float().mean().item() - 0.9) < 0.03
    assert torch.equal(m1, ME.keep_mask(123, 5, 2, 64, 60, 0, 60, 0.1))  # pure function
    assert not torch.equal(m1, ME.keep_mask(123, 6, 2, 64, 60, 0, 60, 0.1))  # new step, new mask
    assert not torch.equal(m1, ME.keep_mask(123, 5, 3, 64, 60, 0, 60, 0.1))  # other buffer
    # a column slice is the same elements of the full mask
    assert torch.equal(m1[:, 30:], ME.keep_mask(123, 5, 2, 64, 60, 30, 30, 0.1))


def test_dropout_reference_is_deterministic_and_trains():
    xs, y = _data(n=200)
    net = _net(drop=0.1)
    opt = FlatAdamW(net.parameters())
    eng = ME.MlpEpoch(ME.splitnn_graph(list(net.bottom_models), net.top_model), opt, 64, seed=3)
    p0 = opt.data.clone()
    stats = []
    for _ in range(6):
        st = torch.zeros(2)
        eng.run(xs, y, st)
        stats.append(st.clone())
    assert not torch.equal(opt.data, p0)
    assert stats[-1][0] < stats[0][0]  # the loss goes down


def test_graph_checks():
    net = _net()
    g = ME.splitnn_graph(list(net.bottom_models), net.top_model)
    assert [b.width for b in g.bufs] == [30, 30, 60, 128, 256, 2] and g.nlev == 5
    assert g.bufs[2].drop == 0.0 and g.bufs[-1].act == "leaky_relu"
    g.layers[0].need_dx = True  # a party input cannot take a gradient
    with pytest.raises(ValueError):
        g.validate()
    # an optimizer over parameters the graph does not train is refused
    extra = torch.nn.Parameter(torch.zeros(3))
    opt = FlatAdamW([*net.parameters(), extra])
    with pytest.raises(ValueError):
        ME.MlpEpoch(ME.splitnn_graph(list(net.bottom_models), net.top_model), opt, 32)
    with pytest.raises(TypeError):
        ME.MlpEpoch(ME.splitnn_graph(list(net.bottom_models), net.top_model),
                    torch.optim.AdamW(net.parameters()), 32)


def test_vfl_network_uses_module_path_on_cpu():
    net = _net()
    assert net.fused_epoch_engine(64) is None  # CPU: torch AdamW, the module path
