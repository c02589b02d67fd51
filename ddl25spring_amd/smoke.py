"""One tiny forward+backward+update of the flagship client-batched ResNet-18 FedAvg step on cuda:0,
plus a check that the in-tree HIP library is what ran."""
from __future__ import annotations

import os

import torch


def run_smoke():
    from .data.images import DeviceImageDataset, synthetic_images
    from .data.split import split
    from .fl.algorithms import FedAvg
    from .models import resnet18_cifar
    from .ops import _lib
    from .runtime import dist as rdist

    assert torch.cuda.is_available(), "smoke() needs cuda:0"
    ctx = rdist.init(device="cuda")
    train = synthetic_images("cifar10", 400, seed=0)
    data = DeviceImageDataset(train, ctx.device)
    parts = split(2, True, 0, labels=train.labels)
    # the headline's reference-precision (fp32) path; DDL_SMOKE_PRECISION=bf16 for the bf16 one
    prec = os.environ.get("DDL_SMOKE_PRECISION", "fp32")
    fl = FedAvg(lambda groups: resnet18_cifar(10, groups=groups, precision=prec), data, parts, lr=0.01,
                batch_size=50, local_epochs=1, client_fraction=1.0, seed=0, eval_every=0, use_graph=True)
    w0 = fl.w_global.clone()
    dt, samples = fl.round()
    torch.cuda.synchronize()
    loss = fl.trainer.last_loss
    assert loss is not None and torch.isfinite(loss).all(), loss
    delta = (fl.w_global - w0).abs().max().item()
    assert delta > 0 and delta == delta, "weights did not move"
    libs = _lib.loaded_library_paths()
    assert any("libddl_kernels.so" in p for p in libs), libs
    print(f"[smoke] resnet18 ({prec}) fedavg round ok: {samples} samples in {dt*1e3:.1f} ms, "
          f"loss={loss.tolist()}, max|dw|={delta:.3e}, native libs={libs}")


if __name__ == "__main__":
    run_smoke()
