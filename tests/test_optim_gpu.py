"""Fused flat Adam/AdamW (one HIP launch) vs torch.optim on device."""
import pytest
import torch

from ddl25spring_amd.models.tabular import HeartDiseaseNN
from ddl25spring_amd.optim import FlatAdam, FlatAdamW

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("decoupled", [False, True])
def test_flat_adam_cuda(cuda, decoupled):
    torch.manual_seed(0)
    a, b = HeartDiseaseNN().to(cuda), HeartDiseaseNN().to(cuda)
    b.load_state_dict(a.state_dict())
    a.dropout.p = b.dropout.p = 0.0
    oa = (FlatAdamW if decoupled else FlatAdam)(a.parameters(), lr=1e-2)
    ob = (torch.optim.AdamW if decoupled else torch.optim.Adam)(b.parameters(), lr=1e-2)
    x, y = torch.randn(64, 30, device=cuda), torch.randint(0, 2, (64,), device=cuda)
    for _ in range(5):
        for m, o in ((a, oa), (b, ob)):
            o.zero_grad()
            torch.nn.functional.cross_entropy(m(x), y).backward()
            o.step()
    for pa, pb in zip(a.parameters(), b.parameters()):
        assert torch.allclose(pa, pb, atol=1e-4, rtol=1e-3)
