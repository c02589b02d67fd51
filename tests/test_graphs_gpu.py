"""HIP-graph replay of torch-style training steps (runtime.graphs.CapturedStep): identical to the
eager steps, and the federated DCGAN's per-client graphs keep each client's Adam step count."""
import pytest
import torch

from ddl25spring_amd.models import tabular as T
from ddl25spring_amd.optim import FlatAdamW
from ddl25spring_amd.runtime.graphs import CapturedStep

pytestmark = pytest.mark.gpu


def _mlp_run(cuda, graph: bool, steps: int = 6):
    torch.manual_seed(0)
    net = torch.nn.Sequential(T.FLinear(30, 64, "leaky_relu"), T.FLinear(64, 2)).to(cuda)
    opt = FlatAdamW(net.parameters())
    crit = T.SoftCrossEntropy()
    g = torch.Generator().manual_seed(1)
    x = torch.randn(96, 30, generator=g).to(cuda)
    y = torch.nn.functional.one_hot(torch.randint(0, 2, (96,), generator=g), 2).float().to(cuda)

    def epoch():
        for b in range(0, 96, 40):  # 40, 40, 16: a short last batch too
            opt.zero_grad()
            loss = crit(net(x[b:b + 40]), y[b:b + 40])
            loss.backward()
            opt.step()
        return loss.detach()

    step = CapturedStep(epoch, warmup=1, enabled=graph)
    for _ in range(steps):
        loss = step()
    torch.cuda.synchronize()
    return opt.data.clone(), loss.clone(), int(opt.t_dev.item())


def test_captured_step_matches_eager(cuda):
    """Warm-up, capture and replays perform one epoch per call, like the eager loop: same
    parameters (Adam's bias correction runs off the device step counter), same last loss."""
    pe, le, te = _mlp_run(cuda, False)
    pg, lg, tg = _mlp_run(cuda, True)
    assert te == tg == 18
    assert ((pg - pe).norm() / pe.norm()).item() < 1e-5
    assert abs(lg.item() - le.item()) < 1e-4


@pytest.mark.parametrize("batched", [False, True])
def test_federated_gan_graphs_keep_client_adam_state(cuda, batched):
    """Two clients, three rounds (eager, capture, replay): finite losses, and each client's
    restored device step counter continues from its own count (3 rounds x 2 local steps). The
    client-batched engine runs a round's 2 clients as ONE graph replay."""
    from ddl25spring_amd.fl.gan import FederatedGAN
    from ddl25spring_amd.models.dcgan import to_nhwc_padded
    torch.manual_seed(0)
    data = [to_nhwc_padded(torch.rand(48, 3, 32, 32) * 2 - 1).to(cuda) for _ in range(2)]
    fg = FederatedGAN(data, ngf=32, ndf=32, local_steps=2, batch_size=8, seed=1, device=cuda, batched=batched)
    assert fg.use_graph
    res = fg.run(3)
    fg.flush_slots()
    if batched:
        assert list(fg._bgraphs) == [2] and fg._bgraphs[2].calls == 3 and fg._bgraphs[2].graph is not None
    assert res.rounds == 3 and res.samples == 3 * 2 * 2 * 8
    assert all(torch.isfinite(torch.tensor(res.loss_d))) and all(torch.isfinite(torch.tensor(res.loss_g)))
    for c in (0, 1):
        st = fg._state[c]
        assert int(st[6].item()) == 6 and int(st[7].item()) == 6, (c, st[6], st[7])
