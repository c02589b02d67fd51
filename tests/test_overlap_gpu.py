"""Backward stream split (weight grads on a side stream, ``Fn.wgrad_overlap``): same gradients as
the single-stream backward, eagerly and replayed from a captured HIP graph."""
import pytest
import torch

from ddl25spring_amd.data.images import DeviceImageDataset, synthetic_images
from ddl25spring_amd.models import mnist_cnn, resnet18_cifar

pytestmark = pytest.mark.gpu


def _grads(cuda, model_fn, kind, overlap: bool, graph: bool):
    arr = synthetic_images(kind, 64, seed=0)
    net = model_fn(groups=2).to(cuda, seed=5)
    net.overlap_wgrad = overlap
    data = DeviceImageDataset(arr, cuda, net.input_spec)
    idx = torch.arange(64, dtype=torch.int32, device=cuda).view(2, 32)
    x, y = data.batch(idx)
    st = net.store
    if not graph:
        st.grad.zero_()
        net.train_step(x, y)
        torch.cuda.synchronize()
        return st.grad.clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        st.grad.zero_()
        net.train_step(x, y)  # eager warm-up (sizes the scratch arena)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        st.grad.zero_()
        net.train_step(x, y)
    for c in net.rng_counters():  # the warm-up advanced the dropout counters: rewind them
        c.zero_()
    g.replay()
    torch.cuda.synchronize()
    return st.grad.clone()


def _rel(a, b):
    return ((a - b).norm() / b.norm()).item()


def test_wgrad_side_stream_exact_without_bn(cuda):
    """MnistCnn (no BatchNorm): only the wgrad split-K atomics reorder -> rounding-level match."""
    ref = _grads(cuda, mnist_cnn, "mnist", False, False)
    assert ref.abs().sum() > 0
    for graph in (False, True):
        assert _rel(_grads(cuda, mnist_cnn, "mnist", True, graph), ref) < 1e-3, graph


def test_wgrad_side_stream_resnet_within_noise_floor(cuda):
    """ResNet-18: BN statistics are fp32 atomics, and at random init their ~1e-7 order noise
    grows through the BN backward chain to ~15% of the bottom layers' gradients between two
    identical single-stream runs. The side-stream run must stay within that same floor."""
    ref = _grads(cuda, resnet18_cifar, "cifar10", False, False)
    floor = _rel(_grads(cuda, resnet18_cifar, "cifar10", False, False), ref)
    for graph in (False, True):
        rel = _rel(_grads(cuda, resnet18_cifar, "cifar10", True, graph), ref)
        assert rel < 1.5 * floor + 0.02, (graph, rel, floor)


def test_cross_block_bn_backward_fusion_within_noise_floor(cuda, monkeypatch):
    """Residual blocks fuse the previous layer's ReLU mask + BN backward reduce into their last
    dgrad epilogue (Net._plan_fusions). Same gradients as the unfused backward, within the
    BN-atomics noise floor of two identical runs."""
    monkeypatch.setenv("DDL_FUSE_BN_BWD", "0")
    ref = _grads(cuda, resnet18_cifar, "cifar10", False, False)
    floor = _rel(_grads(cuda, resnet18_cifar, "cifar10", False, False), ref)
    monkeypatch.setenv("DDL_FUSE_BN_BWD", "1")
    net = resnet18_cifar(groups=2)
    assert sum(bool(layer.fuse_out_bn) for layer in net.layers) == 9  # 8 blocks + the pool
    for graph in (False, True):
        rel = _rel(_grads(cuda, resnet18_cifar, "cifar10", False, graph), ref)
        assert rel < 1.5 * floor + 0.02, (graph, rel, floor)


def test_fused_head_matches_per_layer_head(cuda, monkeypatch):
    """ResNet-18's pool -> fc -> CE -> fc grads -> pool backward (+ the last BN's reduce) in two
    launches (Fn.head_train): the fc gradients match the per-layer path's to bf16 rounding (that
    path rounds the pooled vector, logits and their gradients to bf16), every other gradient
    within the BN-atomics noise floor, eagerly and graph-replayed."""
    from ddl25spring_amd.ops import functional as Fn
    monkeypatch.setattr(Fn, "HEAD_FUSED", False)
    ref = _grads(cuda, resnet18_cifar, "cifar10", False, False)
    floor = _rel(_grads(cuda, resnet18_cifar, "cifar10", False, False), ref)
    monkeypatch.setattr(Fn, "HEAD_FUSED", True)
    net = resnet18_cifar(groups=2)
    lin = net.layers[-1]
    sw, sb = net.store.specs[lin.w], net.store.specs[lin.b]
    fc = slice(sw.offset, sb.offset + sb.numel)
    for graph in (False, True):
        g = _grads(cuda, resnet18_cifar, "cifar10", False, graph)
        assert _rel(g, ref) < 1.5 * floor + 0.02, (graph, _rel(g, ref), floor)
        assert _rel(g[:, fc], ref[:, fc]) < 2e-2, graph
