"""The fused classifier head's CPU path (``Fn.head_train``) against autograd on the same
composition: global average pool -> Linear -> cross-entropy, and the pool backward fused with a
BatchNorm's ReLU mask and backward sums."""
import torch
import torch.nn.functional as F

import ddl25spring_amd.ops.functional as Fn
from ddl25spring_amd.models import resnet18_cifar


def test_head_train_cpu_matches_autograd():
    torch.manual_seed(0)
    G, N, H, W, C, Kp, ncls = 2, 6, 3, 3, 64, 32, 10
    x = torch.randn(G, N, H, W, C).relu().to(torch.bfloat16)
    w = (torch.randn(G, Kp, 1, 1, C) * 0.1).to(torch.bfloat16)
    b = torch.randn(G, Kp) * 0.1
    labels = torch.randint(0, ncls, (G, N), dtype=torch.int32)
    dw, db = torch.zeros(G, Kp, 1, 1, C), torch.zeros(G, Kp)
    loss, correct, dx, part = Fn.head_train(x, w, b, labels, ncls, 1.0 / N, dw, db, with_correct=True)
    assert part is None
    xr = x.float().requires_grad_(True)
    wr = w.float().reshape(G, Kp, C)[:, :ncls].clone().requires_grad_(True)
    br = b[:, :ncls].clone().requires_grad_(True)
    z = torch.einsum("gnc,gkc->gnk", xr.mean((2, 3)), wr) + br[:, None]
    ref = torch.stack([F.cross_entropy(z[g], labels[g].long()) for g in range(G)])
    ref.sum().backward()
    torch.testing.assert_close(loss, ref.detach(), rtol=1e-5, atol=1e-6)
    assert torch.equal(correct, (z.argmax(-1) == labels.long()).sum(1).to(torch.int32))
    torch.testing.assert_close(dw.reshape(G, Kp, C)[:, :ncls], wr.grad, rtol=1e-5, atol=1e-6)
    assert dw.reshape(G, Kp, C)[:, ncls:].abs().max() == 0
    torch.testing.assert_close(db[:, :ncls], br.grad, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(dx.float(), xr.grad, rtol=1e-2, atol=1e-4)
    # with the producing BN fused: masked by x > 0 and its backward sums
    c = torch.randn(G, N, H, W, C).to(torch.bfloat16)
    mean, rstd = torch.randn(G, C) * 0.1, torch.rand(G, C) + 0.5
    dx2, part2 = Fn.head_train(x, w, b, labels, ncls, 1.0 / N, dw * 0, db * 0, bn=(c, mean, rstd))[2:]
    masked = xr.grad * (x.float() > 0)
    torch.testing.assert_close(dx2.float(), masked, rtol=1e-2, atol=1e-4)
    xh = (c.float() - mean[:, None, None, None]) * rstd[:, None, None, None]
    torch.testing.assert_close(part2[:, :, 0].sum(1), dx2.float().sum((1, 2, 3)), rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(part2[:, :, 1].sum(1), (dx2.float() * xh).sum((1, 2, 3)), rtol=1e-4, atol=1e-5)


def test_resnet_head_is_fusable():
    """ResNet-18 ends in pool -> Linear(512 -> 10) with the last block's BN fused into the pool:
    the shapes ``Net._fused_head`` hands to the fused launches on the GPU."""
    net = resnet18_cifar(groups=1)
    pool, lin = net.layers[-2], net.layers[-1]
    assert pool.name == "avgpool" and pool.fuse_out_bn and lin.linear and not lin.bn and not lin.act
    assert Fn.head_train_ok(lin.cin, net.num_classes)
    assert net._fused_head(torch.zeros(1), None, None) is None  # CPU tensors keep the per-layer path
