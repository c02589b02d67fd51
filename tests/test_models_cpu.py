"""Native nets (explicit fwd/bwd over the op layer, CPU reference path) vs torch autograd."""
import pytest
import torch
import torch.nn.functional as F

import ddl25spring_amd.ops.reference as R
from ddl25spring_amd.models import params as P

from ddl25spring_amd.models import convert, mnist_cnn, mnist_mlp, resnet18_cifar
from ddl25spring_amd.models.torch_ref import TorchMLP, TorchMnistCnn, torch_resnet18_cifar
from ddl25spring_amd.models.zoo import mnist_cnn_mapping, mnist_mlp_mapping


def _cos(a, b):
    a, b = a.flatten().double(), b.flatten().double()
    return (a @ b / (a.norm() * b.norm() + 1e-30)).item()


@pytest.fixture
def fp32_emulation(monkeypatch):
    """Run the reference op path without bf16 rounding: checks fwd/bwd logic exactly."""
    monkeypatch.setattr(R, "_bf", lambda t: t.float())
    monkeypatch.setattr(P, "CPU_SHADOW_DTYPE", torch.float32)


def test_resnet18_exact_in_fp32(fp32_emulation):
    torch.manual_seed(0)
    tm = torch_resnet18_cifar(10)
    net = resnet18_cifar(10, groups=1).to("cpu")
    mapping = convert.resnet_mapping(net)
    convert.import_torch(net, tm, mapping)
    x = torch.randn(4, 3, 32, 32)
    y = torch.randint(0, 10, (4,))
    loss_t = F.cross_entropy(tm(x), y)
    loss_t.backward()
    net.store.zero_grad()
    loss, _ = net.train_step(net.prepare_input(x), y[None].to(torch.int32))
    assert abs(loss[0].item() - loss_t.item()) < 1e-4
    g = convert.export_torch(net, tm, mapping, grads=True)
    for name, p in tm.named_parameters():
        assert _cos(g[name], p.grad) > 0.99999, name
        assert (g[name] - p.grad).abs().max() < 1e-3 * (p.grad.abs().max() + 1e-3), name


def test_resnet18_bf16_close_to_torch():
    torch.manual_seed(0)
    tm = torch_resnet18_cifar(10)
    net = resnet18_cifar(10, groups=2).to("cpu")
    mapping = convert.resnet_mapping(net)
    convert.import_torch(net, tm, mapping)
    x = torch.randn(4, 3, 32, 32)
    y = torch.randint(0, 10, (4,))
    # torch oracle (train-mode BN)
    loss_t = F.cross_entropy(tm(x), y)
    loss_t.backward()
    # native: same batch in both client groups
    xin = net.prepare_input(x)
    xin = torch.cat([xin, xin], 0)
    lab = torch.stack([y, y]).to(torch.int32)
    net.store.zero_grad()
    loss, _ = net.train_step(xin, lab)
    assert abs(loss[0].item() - loss_t.item()) < 5e-2 * max(1, loss_t.item())
    assert torch.allclose(loss[0], loss[1])
    g = convert.export_torch(net, tm, mapping, group=1, grads=True)
    for name, p in tm.named_parameters():
        c = _cos(g[name], p.grad)
        assert c > 0.85, (name, c)  # bf16 activations: deep grads of an untrained net drift
    # running stats updated like torch's
    sd = convert.export_torch(net, tm, mapping, group=0)
    assert torch.allclose(sd["layer1.0.bn1.running_mean"], tm.layer1[0].bn1.running_mean, atol=2e-2)


def test_mnist_cnn_torch_compatible_api():
    torch.manual_seed(3)
    tm = TorchMnistCnn()
    net = mnist_cnn().to("cpu")
    convert.import_torch(net, tm, mnist_cnn_mapping())
    net.eval(); tm.eval()
    x = torch.randn(5, 1, 28, 28)
    out = net(x)
    ref = tm(x)
    assert out.shape == (5, 10)
    assert (out - ref).abs().max().item() < 5e-2
    # autograd bridge: reference-style loss.backward() drives the native backward
    net.train(); tm.train()
    for d in [m for m in tm.modules() if isinstance(m, torch.nn.Dropout)]:
        d.p = 0.0
    for layer in net.layers:
        if hasattr(layer, "p"):
            layer.p = 0.0
    y = torch.randint(0, 10, (5,))
    net.zero_grad()
    F.nll_loss(net(x), y).backward()
    F.nll_loss(tm(x), y).backward()
    g = convert.export_torch(net, tm, mnist_cnn_mapping(), grads=True)
    for name, p in tm.named_parameters():
        assert _cos(g[name], p.grad) > 0.98, name


def test_mlp():
    torch.manual_seed(1)
    tm = TorchMLP()
    net = mnist_mlp().to("cpu")
    convert.import_torch(net, tm, mnist_mlp_mapping())
    x = torch.randn(6, 1, 28, 28)
    y = torch.randint(0, 10, (6,))
    F.cross_entropy(tm(x), y).backward()
    net.zero_grad()
    loss, _ = net.train_step(net.prepare_input(x), y[None].to(torch.int32))
    g = convert.export_torch(net, tm, mnist_mlp_mapping(), grads=True)
    for name, p in tm.named_parameters():
        assert _cos(g[name], p.grad) > 0.99, name


def test_rmsnorm_fork_cpu_matches_separate_paths():
    """CPU contract of the LLaMA pre-norm fork: (rmsnorm(x), x), gradients summed over both uses."""
    from ddl25spring_amd.models.llama import LLama  # noqa: F401  (module imports the op)
    from ddl25spring_amd.ops import autograd_ops as A
    torch.manual_seed(0)
    x = torch.randn(2, 5, 16, requires_grad=True)
    g = torch.rand(16) + 0.5
    h, r = A.rmsnorm_fork(x, g)
    assert r is x
    (h * 2 + r * 3).sum().backward()
    x2 = x.detach().clone().requires_grad_(True)
    (A.rmsnorm(x2, g) * 2 + x2 * 3).sum().backward()
    torch.testing.assert_close(x.grad, x2.grad)
