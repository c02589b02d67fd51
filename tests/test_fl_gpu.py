"""The FL engine on the device: HIP-graph replay == eager, learning, robust aggregation, and the
GPU engine against the fp32 CPU engine."""
import pytest
import torch

from ddl25spring_amd.data.images import DeviceImageDataset, synthetic_images
from ddl25spring_amd.data.split import split
from ddl25spring_amd.fl.algorithms import FedAvg, FedSGD
from ddl25spring_amd.fl.attacks import LabelFlip
from ddl25spring_amd.models import mnist_cnn, mnist_mlp
from ddl25spring_amd.runtime.dist import DistContext

pytestmark = pytest.mark.gpu


def _ctx(cuda):
    return DistContext(device=cuda)


@pytest.mark.parametrize("batch,flip", [(50, False), (60, False), (50, True)])
def test_graph_replay_equals_eager(cuda, batch, flip):
    """Captured local steps == eager steps, including dropout: its Philox counter lives on the
    device and advances inside the graph, so every replay draws a fresh mask. batch 60: 200
    samples per client end in a short step of 20, captured in the same graph. flip: a
    label-flipping client (LabelFlip's device-side transform replays inside the graph).

    MnistCnn (no BatchNorm): with BN, the fp32-atomic order noise of the statistics (~1e-7) is
    amplified chaotically by bf16 rounding (two identical eager runs of ResNet-18 differ by ~35%
    of a round's update; the same 1e-7 perturbation does that on the CPU emulation too), which
    would hide a replay bug. Without BN, graph and eager agree to rounding level."""
    arr = synthetic_images("mnist", 800, seed=0)
    parts = split(4, True, 3, labels=arr.labels)
    ws = []
    for graph in (True, False):
        data = DeviceImageDataset(arr, cuda)
        fa = FedAvg(mnist_cnn, data, parts, lr=0.05, batch_size=batch, client_fraction=1.0,
                    seed=3, ctx=_ctx(cuda), use_graph=graph, eval_every=0,
                    attack=LabelFlip([1]) if flip else None)
        w0 = fa.w_global.clone()
        fa.round()
        fa.round()
        ws.append(fa.w_global.clone())
    step = (ws[1] - w0).norm()
    assert step > 0
    assert ((ws[0] - ws[1]).norm() / step).item() < 1e-2


@pytest.mark.parametrize("flip", [False, True])
def test_chunked_round_graph_equals_whole(cuda, monkeypatch, flip):
    """A round longer than GRAPH_MAX_STEPS replays one graph per chunk of steps (a 500-step
    single-client round in one graph segfaulted in hipGraphLaunch). Chunks of 2 steps, the last
    chunk with the short step: same weights as the whole round in one graph."""
    import ddl25spring_amd.fl.local as L
    arr = synthetic_images("mnist", 800, seed=0)
    parts = split(4, True, 3, labels=arr.labels)
    ws = []
    for chunk in (1000, 2):
        monkeypatch.setattr(L, "GRAPH_MAX_STEPS", chunk)
        data = DeviceImageDataset(arr, cuda)
        fa = FedAvg(mnist_cnn, data, parts, lr=0.05, batch_size=60, client_fraction=1.0,
                    seed=3, ctx=_ctx(cuda), use_graph=True, eval_every=0,
                    attack=LabelFlip([1]) if flip else None)
        w0 = fa.w_global.clone()
        fa.round()
        fa.round()
        ws.append(fa.w_global.clone())
    step = (ws[1] - w0).norm()
    assert step > 0
    assert ((ws[0] - ws[1]).norm() / step).item() < 1e-2


def test_fedavg_mnist_cnn_learns_on_device(cuda):
    arr = synthetic_images("mnist", 3000, seed=0)
    tarr = synthetic_images("mnist", 1000, seed=1)
    parts = split(10, True, 10, labels=arr.labels)
    fa = FedAvg(mnist_cnn, DeviceImageDataset(arr, cuda), parts, lr=0.05, batch_size=50,
                client_fraction=0.5, seed=10, ctx=_ctx(cuda), test_data=DeviceImageDataset(tarr, cuda))
    res = fa.run(3)
    assert res.test_accuracy[-1] > 40.0 and res.test_accuracy[-1] >= res.test_accuracy[0], res.test_accuracy
    assert res.message_count == [10, 20, 30]
    assert set(res.phase_ms[-1]) >= {"download", "local_train", "aggregate"}


@pytest.mark.parametrize("algo", [FedAvg, FedSGD])
def test_device_engine_tracks_cpu_engine(cuda, algo):
    """Same protocol, same seeds: the bf16-MFMA device run stays close to the CPU run (an MLP:
    no dropout, whose CPU reference draws its masks from a different generator)."""
    arr = synthetic_images("mnist", 600, seed=0)
    parts = split(4, True, 1, labels=arr.labels)
    kw = dict(lr=0.05, client_fraction=0.5, seed=1)
    if algo is FedAvg:
        kw["batch_size"] = 50
    runs = []
    for dev in (torch.device("cpu"), cuda):
        fa = algo(mnist_mlp, DeviceImageDataset(arr, dev), parts, ctx=DistContext(device=dev), **kw)
        fa.round()
        runs.append(fa.w_global.float().cpu())
    cpu, gpu = runs
    rel = ((cpu - gpu).norm() / cpu.norm()).item()
    assert rel < 2e-2, rel


@pytest.mark.parametrize("agg", ["median", "trimmed_mean", "krum"])
def test_robust_aggregation_on_device(cuda, agg):
    from ddl25spring_amd.fl import aggregate as A
    torch.manual_seed(0)
    honest = torch.randn(1, 5000) * 0.1 + 1.0 + 0.05 * torch.randn(7, 5000)
    rows = torch.cat([honest, -10.0 * torch.ones(2, 5000)])
    a = A.make_aggregator(agg, trim=2, f=2)
    out_gpu = a(DistContext(device=cuda), rows.to(cuda), [9], 5000).cpu()
    out_cpu = a(DistContext(), rows, [9], 5000)
    assert torch.allclose(out_gpu, out_cpu, atol=1e-5)
    assert (out_gpu - honest.mean(0)).abs().max() < 0.3


@pytest.mark.parametrize("agg", ["median", "trimmed_mean", "krum"])
def test_robust_aggregation_k100_native(cuda, agg):
    """K = 100 clients (the Byzantine bench scale) on the native kernels, 20 sign-flip attackers."""
    from ddl25spring_amd.fl import aggregate as A
    torch.manual_seed(1)
    P = 40_000
    center = torch.randn(P) * 0.1
    honest = center + 0.05 * torch.randn(80, P)
    rows = torch.cat([honest, -5.0 * center.expand(20, P)])
    a = A.make_aggregator(agg, trim=0.2, f=20)
    out_gpu = a(DistContext(device=cuda), rows.to(cuda), [100], P).cpu()
    out_cpu = a(DistContext(), rows, [100], P)
    assert torch.allclose(out_gpu, out_cpu, atol=1e-5)
    ref = honest.mean(0)
    # the plain mean is dragged to ~1.2x |ref| away; the coordinate rules keep a small trimming
    # bias (20 of the trimmed values per side are honest), Krum returns one honest client
    assert ((rows.mean(0) - ref).norm() / ref.norm()).item() > 1.0
    # (Krum returns ONE honest client: its own noise, 0.05 * sqrt(P) / |ref| ~ 0.5, remains)
    assert ((out_gpu - ref).norm() / ref.norm()).item() < (0.6 if agg == "krum" else 0.3)
    if agg == "krum":
        assert max(a.last_selected) < 80  # picked an honest client


@pytest.mark.parametrize("model", ["mnist_cnn", "resnet18"])
def test_direct_sgd_equals_gradient_sgd(cuda, model, monkeypatch):
    """Direct SGD (the conv WGRAD launches add -lr * dW into the master weights; one launch then
    refreshes the shadow and steps BN / head params) == zeroed gradients + fused SGD, one
    graph-replayed local step. The two differ only by fp32 rounding (p + sum(-lr * partial) vs
    p - lr * sum(partial)). MnistCnn: 2e-4 of the update (measured with a one-off script, r2). ResNet-18: two
    identical gradient-SGD runs already differ by ~16% of one step's update (fp32-atomic order of
    the BN statistics, amplified through bf16 activations and the BN backward), and direct SGD
    sits at that same noise floor, so it is checked against a second gradient-SGD run."""
    import ddl25spring_amd.fl.local as L
    from ddl25spring_amd.models import resnet18_cifar
    if model == "mnist_cnn":
        arr, fn, modes = synthetic_images("mnist", 100, seed=0), mnist_cnn, (False, True)
    else:
        arr, fn, modes = synthetic_images("cifar10", 100, seed=0), resnet18_cifar, (False, True, False)
    parts = split(2, True, 3, labels=arr.labels)  # 50 samples each: one step of B = 50
    ws = []
    for direct in modes:
        monkeypatch.setattr(L, "DIRECT_SGD", direct)
        fa = FedAvg(fn, DeviceImageDataset(arr, cuda), parts, lr=0.05, batch_size=50,
                    client_fraction=1.0, seed=3, ctx=_ctx(cuda), use_graph=True, eval_every=0)
        w0 = fa.w_global.clone()
        fa.round()
        assert fa.trainer.direct == direct
        ws.append(fa.w_global.clone())
        st = fa.net.store
        assert torch.equal(st.shadow, st.data.to(torch.bfloat16))
        if direct:
            assert torch.count_nonzero(st.grad[:, (st.direct_map == 0).repeat_interleave(16)]) == 0
    step = (ws[0] - w0).norm()
    assert step > 0
    rel = ((ws[0] - ws[1]).norm() / step).item()
    if model == "mnist_cnn":
        assert rel < 2e-3
    else:
        noise = ((ws[0] - ws[2]).norm() / step).item()
        assert rel < 2 * noise + 1e-2, (rel, noise)


def test_unsynchronised_rounds_match_on_device(cuda, monkeypatch):
    """Rounds enqueued back to back without host <-> device syncs (pinned, double-buffered plan
    uploads; bench.py's timed mode) train as the synchronised rounds: same kernels in the same
    order. Checked tightly with deterministic plans (no autotuner, gradient buffer + fused SGD, one
    split-K slice per WGRAD tile):
    scripts/fl_sync_diag.py (profiles/fl_sync_diag_r5e.txt) found the bf16 run-to-run spread
    (~1e-2 of a round's update, synchronised runs included) to come from the WGRAD launches, whose
    split-K partials meet through fp32 atomics (into the master weights with direct SGD, into the
    gradient buffer without), amplified by bf16 shadow rounding — not from the unsynchronised path."""
    from ddl25spring_amd.fl import local
    from ddl25spring_amd.ops import autotune
    from ddl25spring_amd.ops import functional as Fn
    monkeypatch.setattr(autotune, "ENABLED", False)
    monkeypatch.setattr(autotune, "_CACHE", {})
    monkeypatch.setattr(local, "DIRECT_SGD", False)
    # the bf16 WGRAD's split-K slices meet through fp32 atomics: one slice per output tile makes
    # the step deterministic (two synchronised runs still drifted 2e-4 apart with split-K)
    wgrad = Fn.conv_wgrad
    monkeypatch.setattr(Fn, "conv_wgrad", lambda *a, **k: wgrad(*a, **{**k, "splits": 1}))
    arr = synthetic_images("mnist", 800, seed=0)
    parts = split(4, True, 3, labels=arr.labels)
    ws = []
    for sync in (True, False, True):
        fa = FedAvg(mnist_cnn, DeviceImageDataset(arr, cuda), parts, lr=0.05, batch_size=50,
                    client_fraction=1.0, seed=3, ctx=_ctx(cuda), eval_every=0)
        w0 = fa.w_global.clone()
        fa.round()  # capture
        fa.sync_rounds = sync
        for _ in range(3):
            _, s = fa.round()
            assert s == 800
        torch.cuda.synchronize()
        ws.append(fa.w_global.clone())
    step = (ws[0] - w0).norm()
    assert ((ws[0] - ws[2]).norm() / step).item() < 1e-4
    assert ((ws[0] - ws[1]).norm() / step).item() < 1e-4


class _BothAttacks:
    """label flip for some clients + sign flip for others (benchmarks/bench_byzantine.py)."""

    def __init__(self, model_attack, data_attack):
        self.m, self.d = model_attack, data_attack

    def label_transform_for(self, mine, ncls):
        return self.d.label_transform_for(mine, ncls)

    def skip_training(self, c):
        return False

    def poison_updates(self, rows, w_global, mine):
        self.m.poison_updates(rows, w_global, mine)


@pytest.mark.parametrize("agg", ["mean", "median"])
def test_attacked_fp32_graph_unsynced_equals_eager_bitwise(cuda, agg):
    """The Byzantine bench's configuration at fp32 (deterministic kernels, BN included): label-flip
    + sign-flip attackers, rounds replayed from the captured round graph AND enqueued without host
    syncs give exactly the eager synchronised rounds' server model."""
    import functools
    from ddl25spring_amd.fl.attacks import make_attack
    from ddl25spring_amd.models import resnet18_cifar
    arr = synthetic_images("cifar10", 400, seed=0)
    parts = split(4, True, 3, labels=arr.labels)
    ws = []
    for graph, sync in ((False, True), (True, False)):
        fa = FedAvg(functools.partial(resnet18_cifar, precision="fp32"), DeviceImageDataset(arr, cuda), parts,
                    lr=0.02, batch_size=50, client_fraction=1.0, seed=3, ctx=_ctx(cuda), use_graph=graph,
                    eval_every=0, aggregator=agg,
                    attack=_BothAttacks(make_attack("sign_flip", [2]), make_attack("label_flip", [0])))
        fa.sync_rounds = sync
        for _ in range(3):
            fa.round()
        torch.cuda.synchronize()
        ws.append(fa.w_global.clone())
    assert torch.isfinite(ws[0]).all()
    assert torch.equal(ws[0], ws[1])
