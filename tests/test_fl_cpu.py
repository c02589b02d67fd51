"""Horizontal-FL behaviour on the CPU reference path (+ gloo multi-process for the distributed
aggregation). Mirrors the reference's algorithmic invariants."""
import os
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

import ddl25spring_amd.ops.reference as R
from ddl25spring_amd.data.images import DeviceImageDataset, synthetic_images
from ddl25spring_amd.data.split import plan_epoch, split
from ddl25spring_amd.fl import aggregate as A
from ddl25spring_amd.fl.algorithms import FedAvg, FedSGD, FedSgdWeight
from ddl25spring_amd.fl.attacks import LabelFlip, SignFlip
from ddl25spring_amd.models import mnist_mlp
from ddl25spring_amd.models import params as P
from ddl25spring_amd.runtime.dist import DistContext


@pytest.fixture
def fp32(monkeypatch):
    monkeypatch.setattr(R, "_bf", lambda t: t.float())
    monkeypatch.setattr(P, "CPU_SHADOW_DTYPE", torch.float32)


def _data(n=600, seed=0):
    arr = synthetic_images("mnist", n, seed=seed)
    return arr, DeviceImageDataset(arr, "cpu")


def test_split_matches_reference_semantics():
    labels = np.random.default_rng(0).integers(0, 10, 1000)
    iid = split(7, True, 10, labels=labels)
    rng = np.random.default_rng(10)
    ref = np.array_split(rng.permutation(1000), 7)
    assert all(np.array_equal(a, b) for a, b in zip(iid, ref))
    non = split(5, False, 3, labels=labels)
    rng = np.random.default_rng(3)
    shards = np.array_split(np.argsort(labels), 10)
    order = rng.permutation(10).reshape(5, 2)
    for got, pair in zip(non, order):
        assert np.array_equal(got, np.concatenate([shards[i] for i in pair]))
    assert sorted(np.concatenate(non).tolist()) == list(range(1000))


def test_native_epoch_planner():
    idx = [np.arange(10) + 100 * g for g in range(3)]
    plan = plan_epoch(idx, 4, [1, 2, 3])
    assert plan.shape == (3, 3, 4)
    for g in range(3):
        seen = plan[:, g][plan[:, g] >= 0]
        assert sorted(seen.tolist()) == idx[g].tolist()
    assert (plan[-1, :, 2:] == -1).all()


def test_mean_aggregator_equals_weighted_mean():
    ctx = DistContext()
    rows = torch.randn(5, 33)
    coeffs = torch.tensor([0.1, 0.2, 0.3, 0.25, 0.15])
    out = torch.empty(33)
    A.MeanAggregator()(ctx, rows, coeffs, out)
    assert torch.allclose(out, (coeffs[:, None] * rows).sum(0), atol=1e-6)
    A.MeanAggregator()(ctx, rows, torch.full((5,), 0.2), out)
    assert torch.allclose(out, rows.mean(0), atol=1e-6)


@pytest.mark.parametrize("agg", ["median", "trimmed_mean", "krum"])
def test_robust_aggregators_resist_sign_flip(agg):
    torch.manual_seed(0)
    ctx = DistContext()
    honest = torch.randn(1, 200) * 0.1 + 1.0 + 0.05 * torch.randn(7, 200)
    bad = -10.0 * torch.ones(2, 200)
    rows = torch.cat([honest, bad])
    a = A.make_aggregator(agg, trim=2, f=2)
    out = a(ctx, rows, [9], 200)
    assert (out - honest.mean(0)).abs().max() < 0.3, agg
    mean = rows.mean(0)
    assert (mean - honest.mean(0)).abs().max() > 2.0  # the plain mean is wrecked
    if agg == "krum":
        assert all(i < 7 for i in a.last_selected)


def test_fedavg_learns_and_reports(fp32):
    arr, data = _data(600)
    tarr, tdata = _data(300, seed=1)
    parts = split(6, True, 10, labels=arr.labels)
    fa = FedAvg(mnist_mlp, data, parts, lr=0.1, batch_size=50, local_epochs=1, client_fraction=0.5,
                seed=10, test_data=tdata)
    res = fa.run(4)
    assert res.message_count == [6, 12, 18, 24]
    assert res.test_accuracy[-1] > 40.0, res.test_accuracy
    df = res.as_df()
    assert list(df.columns) == ["Round", "Algorithm", "N", "C", "B", "E", "η", "Seed",
                                "Message count", "Test accuracy"]


def test_fedsgd_gradient_equals_fedsgd_weight(fp32):
    """sum_k p_k (w - lr g_k) = w - lr sum_k p_k g_k : the exchanged quantity does not matter."""
    arr, data = _data(400)
    parts = split(4, True, 1, labels=arr.labels)
    kw = dict(lr=0.05, client_fraction=0.5, seed=3)
    g = FedSGD(mnist_mlp, data, parts, **kw)
    w = FedSgdWeight(mnist_mlp, data, parts, **kw)
    for _ in range(2):
        g.round()
        w.round()
    assert torch.allclose(g.w_global, w.w_global, atol=1e-5), (g.w_global - w.w_global).abs().max()


def test_label_flip_attack_hurts_and_median_helps(fp32):
    arr, data = _data(800)
    tarr, tdata = _data(300, seed=1)
    parts = split(8, True, 5, labels=arr.labels)
    bad = [0, 1]
    kw = dict(lr=0.1, batch_size=50, local_epochs=1, client_fraction=1.0, seed=5, test_data=tdata)
    clean = FedAvg(mnist_mlp, data, parts, **kw).run(5).test_accuracy[-1]
    attacked = FedAvg(mnist_mlp, data, parts, attack=SignFlip(bad, scale=4.0), **kw).run(5).test_accuracy[-1]
    assert attacked < clean - 30, (clean, attacked)
    for agg in ("median", "trimmed_mean"):
        defended = FedAvg(mnist_mlp, data, parts, attack=SignFlip(bad, scale=4.0), aggregator=agg,
                          agg_kwargs={"trim": 2}, **kw).run(5).test_accuracy[-1]
        assert defended > attacked + 30, (agg, attacked, defended)
    lf = FedAvg(mnist_mlp, data, parts, attack=LabelFlip(bad), **kw).run(2)
    assert len(lf.test_accuracy) == 2


# --------------------------------------------------------------------------- distributed (gloo)
def _dist_worker(rank, world, port, out_dir, agg):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    R._bf = lambda t: t.float()
    P.CPU_SHADOW_DTYPE = torch.float32
    from ddl25spring_amd.runtime import dist as rdist
    ctx = rdist.init(backend="gloo", device="cpu")
    arr, data = _data(400)
    parts = split(4, True, 7, labels=arr.labels)
    fa = FedAvg(mnist_mlp, data, parts, lr=0.1, batch_size=50, client_fraction=1.0, seed=7,
                ctx=ctx, aggregator=agg)
    fa.round()
    fa.round()
    torch.save(fa.w_global, os.path.join(out_dir, f"w{rank}.pt"))
    rdist.shutdown()


@pytest.mark.parametrize("agg", ["mean", "median", "trimmed_mean", "krum"])
def test_distributed_fedavg_matches_single_process(fp32, agg):
    """2 gloo ranks x 2 clients vs one process holding the 4: the coordinate-sharded rules go through
    pack_shards + all-to-all + all-gather at world 2 and read the rows in place at world 1."""
    arr, data = _data(400)
    parts = split(4, True, 7, labels=arr.labels)
    single = FedAvg(mnist_mlp, data, parts, lr=0.1, batch_size=50, client_fraction=1.0, seed=7,
                    ctx=DistContext(), aggregator=agg)
    single.round()
    single.round()
    with tempfile.TemporaryDirectory() as d:
        port = 29600 + (os.getpid() % 200) + 10 * ["mean", "median", "trimmed_mean", "krum"].index(agg)
        mp.spawn(_dist_worker, args=(2, port, d, agg), nprocs=2, join=True)
        w0 = torch.load(os.path.join(d, "w0.pt"), weights_only=True)
        w1 = torch.load(os.path.join(d, "w1.pt"), weights_only=True)
    assert torch.equal(w0, w1)  # replicated server state stays identical on every rank
    assert torch.allclose(w0, single.w_global, atol=1e-5), (w0 - single.w_global).abs().max()


@pytest.mark.parametrize("algo", [FedAvg, FedSGD])
def test_checkpoint_resume_is_identical(fp32, algo):
    from ddl25spring_amd.fl import checkpoint as ckpt
    arr, data = _data(400)
    parts = split(6, True, 10, labels=arr.labels)
    kw = dict(lr=0.05, batch_size=50, client_fraction=0.5, seed=4, dropout=0.2)
    ref = algo(mnist_mlp, data, parts, **kw)
    ref.run(4)
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "fl.pt")
        a = algo(mnist_mlp, data, parts, **kw)
        res = ckpt.run_with_checkpoints(a, 2, path)
        assert len(res.message_count) == 2
        b = algo(mnist_mlp, data, parts, **kw)  # fresh process-equivalent: rebuild, then resume
        res = ckpt.run_with_checkpoints(b, 4, path)
        assert res.message_count == [6, 12, 18, 24] and b.round_idx == 4
    assert torch.equal(b.w_global, ref.w_global)
    assert b.dropped == ref.dropped


def test_client_dropout_keeps_sampling_stream(fp32):
    arr, data = _data(400)
    parts = split(8, True, 10, labels=arr.labels)
    kw = dict(lr=0.05, batch_size=50, client_fraction=0.5, seed=5)
    full = FedAvg(mnist_mlp, data, parts, **kw)
    drop = FedAvg(mnist_mlp, data, parts, dropout=0.5, **kw)
    for _ in range(3):
        full.round()
        drop.round()
    assert full.rng.bit_generator.state == drop.rng.bit_generator.state
    assert sum(len(d) for d in drop.dropped) > 0
    total = FedAvg(mnist_mlp, data, parts, dropout=1.0, **kw)
    w0 = total.w_global.clone()
    dt, samples = total.round()
    assert samples == 0 and torch.equal(total.w_global, w0)


def test_free_rider_does_not_stall_honest_clients(fp32):
    """A sampled free rider must not stop the honest clients of the same GPU from training."""
    from ddl25spring_amd.fl.attacks import FreeRider
    arr, data = _data(600)
    parts = split(6, True, 10, labels=arr.labels)
    kw = dict(lr=0.1, batch_size=50, client_fraction=1.0, seed=10)
    fa = FedAvg(mnist_mlp, data, parts, attack=FreeRider([0]), **kw)
    w0 = fa.w_global.clone()
    dt, samples = fa.round()
    assert samples == 500  # 5 honest clients x 100 samples (the free rider's work is not counted)
    assert (fa.w_global - w0).abs().max() > 1e-3
    # the free rider's row is the server model: FedAvg == honest-only FedAvg scaled by 5/6
    clean = FedAvg(mnist_mlp, data, parts, **kw)
    clean.round()
    st = clean.net.store
    upd = (st.data[:6] - w0)
    mine, _ = clean._assign(np.random.default_rng(10).choice(6, 6, replace=False))
    keep = torch.tensor([c != 0 for c in mine])
    expect = w0 + upd[keep].sum(0) / 6
    assert torch.allclose(fa.w_global, expect, atol=1e-5)


def test_torch_planner_matches_dataloader_shuffle():
    """planner='torch' yields exactly DataLoader(shuffle=True, generator=g)'s batches, epoch after
    epoch with the same generator (as WeightClient.update runs E epochs)."""
    from torch.utils.data import DataLoader
    from ddl25spring_amd.fl.local import LocalTrainer
    n, B = 23, 5
    ci = np.arange(100, 100 + n)
    dl = DataLoader(torch.utils.data.TensorDataset(torch.as_tensor(ci)), batch_size=B,
                    shuffle=True, generator=torch.Generator().manual_seed(5))
    want = [[b[0].tolist() for b in dl] for _ in range(2)]
    tr = LocalTrainer.__new__(LocalTrainer)
    tr.B = B
    gen = torch.Generator().manual_seed(5)
    for ep in range(2):
        plan = tr._torch_plan([ci], [gen])
        got = [[int(v) for v in plan[s, 0] if v >= 0] for s in range(plan.shape[0])]
        assert got == want[ep], ep
    first = plan_epoch([ci], B, [5], True, "torch")
    assert [[int(v) for v in first[s, 0] if v >= 0] for s in range(first.shape[0])] == want[0]


def test_label_transform_graph_policy(fp32):
    """LabelFlip's transform is pure device ops with a graph_key: its rounds stay graph-replayed
    (the key tells the trainer which captured round fits). A transform without one runs that
    round eagerly, and later rounds without a transform get the graphs back."""
    from ddl25spring_amd.fl.attacks import Attack
    arr, data = _data(400)
    parts = split(4, True, 3, labels=arr.labels)
    fa = FedAvg(mnist_mlp, data, parts, lr=0.05, batch_size=50, client_fraction=1.0, seed=3,
                attack=LabelFlip([1]), use_graph=True)
    tr = fa._trainer([0, 1])
    assert tr.label_transform.graph_key == ("label_flip", 2, 10)
    assert tr.use_graph == fa._graph_default
    tr = fa._trainer([0, 2])
    assert tr.label_transform is None and tr.use_graph == fa._graph_default

    class Custom(Attack):
        def label_transform_for(self, slot_clients, num_classes):
            return lambda y, g0, g1: y

    fa.attack = Custom([1])
    tr = fa._trainer([0, 1])
    assert tr.label_transform is not None and tr.use_graph is False
    fa.attack = None
    assert fa._trainer([0, 1]).use_graph == fa._graph_default


def test_checkpoint_resume_under_gaussian_attack(fp32):
    from ddl25spring_amd.fl import checkpoint as ckpt
    from ddl25spring_amd.fl.attacks import GaussianNoise
    arr, data = _data(400)
    parts = split(4, True, 2, labels=arr.labels)
    kw = dict(lr=0.05, batch_size=50, client_fraction=1.0, seed=2)
    ref = FedAvg(mnist_mlp, data, parts, attack=GaussianNoise([1], sigma=0.1, seed=9), **kw)
    ref.run(3)
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "fl.pt")
        a = FedAvg(mnist_mlp, data, parts, attack=GaussianNoise([1], sigma=0.1, seed=9), **kw)
        ckpt.run_with_checkpoints(a, 2, path)
        b = FedAvg(mnist_mlp, data, parts, attack=GaussianNoise([1], sigma=0.1, seed=9), **kw)
        ckpt.run_with_checkpoints(b, 3, path)
    assert torch.equal(b.w_global, ref.w_global)


@pytest.mark.parametrize("model", ["mnist_cnn", "resnet_tiny"])
def test_direct_sgd_matches_gradient_sgd(fp32, model):
    """Direct SGD (conv WGRAD adds -lr*dW straight into the master weights, then one launch
    refreshes the shadow and steps the non-conv params) == zero grads + backward + fused SGD."""
    from ddl25spring_amd.fl.local import LocalTrainer
    from ddl25spring_amd.models import mnist_cnn
    from ddl25spring_amd.models.resnet import BasicBlock, _resnet
    if model == "mnist_cnn":
        arr, data = _data(120)
        make = mnist_cnn
    else:
        arr = synthetic_images("cifar10", 48, seed=0)
        data = DeviceImageDataset(arr, "cpu")
        make = lambda groups: _resnet(BasicBlock, (1, 1, 0, 0), 10, groups, "cifar")  # noqa: E731
    parts = split(2, True, 10, labels=arr.labels)
    out = []
    for direct in (False, True):
        net = make(groups=2).to("cpu", seed=3)
        data.set_input_spec(net.input_spec)
        assert 0 < net.store.n_direct < net.store.P
        # flat layout stays in declaration order (the DP bucketer and flat checkpoints rely on it)
        offs = [o for _, o, _ in net.store.param_layout()]
        assert offs == sorted(offs)
        tr = LocalTrainer(net, data, 0.05, 8, use_graph=False, direct=direct)
        assert tr.direct == direct
        tr.run([np.asarray(p) for p in parts], [11, 12], epochs=1)
        out.append((net.store.data.clone(), net.store.shadow.clone(), net.store.grad.clone()))
    (w0, s0, g0), (w1, s1, g1) = out
    assert torch.allclose(w0, w1, atol=1e-5, rtol=1e-4), (w0 - w1).abs().max()
    assert torch.allclose(s1, w1.to(s1.dtype))
    rest = (net.store.direct_map == 0).repeat_interleave(16)
    assert torch.count_nonzero(g1[:, rest]) == 0  # non-direct grads left zeroed for the next step


def test_checkpoint_layout_remap(fp32):
    """Flat checkpoints carry their parameter layout and are remapped by name: a checkpoint whose
    flat rows use another layout (here: the parameters in reverse order) resumes to the same
    model."""
    from ddl25spring_amd.models import mnist_cnn
    arr, data = _data(200)
    parts = split(2, True, 10, labels=arr.labels)
    kw = dict(lr=0.05, batch_size=50, client_fraction=1.0, seed=4)
    fa = FedAvg(mnist_cnn, data, parts, **kw)
    fa.run(1)
    st = fa.net.store
    sd = fa.state_dict()
    other = dict(sd)
    flat, layout, off = torch.zeros_like(sd["w_global"]), [], 0
    for name, o, n in reversed(st.param_layout()):
        flat[off:off + n] = sd["w_global"][o:o + n]
        layout.append([name, off, n])
        off += (n + 15) // 16 * 16
    other["w_global"], other["param_layout"] = flat, layout
    for ck in (sd, other):
        fb = FedAvg(mnist_cnn, data, parts, **kw)
        fb.load_state_dict(ck)
        assert torch.equal(fb.w_global, fa.w_global)


def test_stragglers_deadline_policy(fp32):
    """Straggler injection: without a deadline every sampled client reports and the simulated round
    time is the slowest one (straggler_slowdown x nominal); with a deadline below the slowdown the
    stragglers are dropped from aggregation, on their own RNG stream (client sampling unchanged),
    and the state resumes exactly."""
    arr, data = _data(300)
    parts = split(6, True, 10, labels=arr.labels)
    kw = dict(lr=0.05, batch_size=50, client_fraction=1.0, seed=4)
    base = FedAvg(mnist_mlp, data, parts, **kw)
    slow = FedAvg(mnist_mlp, data, parts, stragglers=0.5, straggler_slowdown=4.0, **kw)
    cut = FedAvg(mnist_mlp, data, parts, stragglers=0.5, straggler_slowdown=4.0, deadline=2.0, **kw)
    for fa in (base, slow, cut):
        fa.run(3)
    assert torch.equal(base.w_global, slow.w_global)  # no deadline: same aggregation
    assert slow.straggled == [[], [], []] and max(slow.sim_time) == pytest.approx(4.0)
    n_late = sum(len(s) for s in cut.straggled)
    assert n_late > 0 and max(cut.sim_time) == pytest.approx(1.0)
    assert not torch.equal(base.w_global, cut.w_global)
    again = FedAvg(mnist_mlp, data, parts, stragglers=0.5, straggler_slowdown=4.0, deadline=2.0, **kw)
    again.run(2)
    resumed = FedAvg(mnist_mlp, data, parts, stragglers=0.5, straggler_slowdown=4.0, deadline=2.0, **kw)
    resumed.load_state_dict(again.state_dict())
    resumed.run(1)
    assert resumed.straggled == cut.straggled and torch.equal(resumed.w_global, cut.w_global)


def test_unsynchronised_rounds_match(fp32):
    """sync_rounds=False (no host <-> device sync inside a round, the throughput mode of bench.py)
    trains exactly as the synchronised rounds; round() then reports this rank's samples."""
    arr, data = _data(300)
    parts = split(6, True, 10, labels=arr.labels)
    kw = dict(lr=0.05, batch_size=50, client_fraction=0.5, seed=4)
    a, b = FedAvg(mnist_mlp, data, parts, **kw), FedAvg(mnist_mlp, data, parts, **kw)
    b.sync_rounds = False
    for _ in range(3):
        _, sa = a.round()
        dt, sb = b.round()
        assert dt == 0.0 and sa == sb
    assert torch.equal(a.w_global, b.w_global)
