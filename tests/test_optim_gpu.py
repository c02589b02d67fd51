"""Fused flat Adam/AdamW (one HIP launch) vs torch.optim on device.

A quadratic objective keeps every gradient well away from zero: Adam normalises g/sqrt(v), so on
near-zero gradients (dead units of a real net) 1-ulp differences flip whole +-lr steps, which says
nothing about the kernel."""
import pytest
import torch

from ddl25spring_amd.optim import FlatAdam, FlatAdamW

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("decoupled", [False, True])
def test_flat_adam_cuda(cuda, decoupled):
    torch.manual_seed(0)
    shapes = [(64, 30), (64,), (7, 3, 5), (1000,)]
    a = [torch.nn.Parameter(torch.randn(s, device=cuda)) for s in shapes]
    b = [torch.nn.Parameter(p.detach().clone()) for p in a]
    tgt = [torch.randn(s, device=cuda) for s in shapes]
    oa = (FlatAdamW if decoupled else FlatAdam)(a, lr=1e-2, weight_decay=0.05)
    ob = (torch.optim.AdamW if decoupled else torch.optim.Adam)(b, lr=1e-2, weight_decay=0.05)
    for _ in range(10):
        for ps, o in ((a, oa), (b, ob)):
            o.zero_grad()
            sum(((p - t) ** 2 * (1 + i)).sum() for i, (p, t) in enumerate(zip(ps, tgt))).backward()
            o.step()
    for pa, pb in zip(a, b):
        assert torch.allclose(pa, pb, atol=1e-5, rtol=1e-5)
