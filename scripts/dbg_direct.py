"""Per-parameter diff of direct SGD vs gradient SGD on the device (LocalTrainer, one or more steps),
against the run-to-run noise floor of two identical gradient-SGD runs."""
import sys

import numpy as np
import torch
from ddl25spring_amd.data.images import DeviceImageDataset, synthetic_images
from ddl25spring_amd.data.split import split
from ddl25spring_amd.fl.local import LocalTrainer
from ddl25spring_amd.models import mnist_cnn, resnet18_cifar

dev = torch.device("cuda", 0)
model = sys.argv[1] if len(sys.argv) > 1 else "mnist"
fn, kind = (mnist_cnn, "mnist") if model == "mnist" else (resnet18_cifar, "cifar10")
arr = synthetic_images(kind, 800, seed=0)
data = DeviceImageDataset(arr, dev)
parts = split(2, True, 3, labels=arr.labels)
for graph, n in ((False, 50), (True, 50), (True, 200)):
    nets = []
    for direct in (False, False, True):
        net = fn(groups=2).to(dev, seed=3)
        data.set_input_spec(net.input_spec)
        w0 = net.store.data.clone()
        tr = LocalTrainer(net, data, 0.05, 50, use_graph=graph, direct=direct)
        tr.run([np.asarray(p)[:n] for p in parts], [11, 12], epochs=1)
        torch.cuda.synchronize()
        nets.append(net)
    s0, s1, s2 = (n_.store.data for n_ in nets)
    step = (s0 - w0).norm().item()
    print(f"graph={graph} samples={n}: |step|={step:.3e} noise(grad vs grad)={(s0 - s1).norm().item() / step:.3e}"
          f" direct vs grad={(s0 - s2).norm().item() / step:.3e}")
    worst = []
    for name, s in nets[0].store.specs.items():
        if s.buffer:
            continue
        a, b, c = (n_.store.param(name) for n_ in nets)
        d0 = (a - nets[0].store._view(w0, s)).norm().item() + 1e-30
        worst.append(((a - c).norm().item() / d0, (a - b).norm().item() / d0, name, s.direct))
    for r in sorted(worst, reverse=True)[:6]:
        print(f"   {r[2]:34s} direct={r[3]} rel diff direct {r[0]:.3e}  noise {r[1]:.3e}")
