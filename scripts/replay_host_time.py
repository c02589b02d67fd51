"""Host time of the round graph's replay() and of a whole unsynchronised round (1-client bench
shape): does the host run ahead of the GPU, or does the launch block?"""
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from ddl25spring_amd.data.images import DeviceImageDataset, synthetic_images  # noqa: E402
from ddl25spring_amd.data.split import split  # noqa: E402
from ddl25spring_amd.fl import local as L  # noqa: E402
from ddl25spring_amd.fl.algorithms import FedAvg  # noqa: E402
from ddl25spring_amd.models import resnet18_cifar  # noqa: E402
from ddl25spring_amd.runtime import dist as rdist  # noqa: E402

ctx = rdist.init()
times = []
orig = L.LocalTrainer._graph_run


def timed(self, *a, **k):
    t = time.perf_counter()
    r = orig(self, *a, **k)
    times.append(time.perf_counter() - t)
    return r


L.LocalTrainer._graph_run = timed
train = synthetic_images("cifar10", 6250, seed=0)
fl = FedAvg(resnet18_cifar, DeviceImageDataset(train, ctx.device), split(1, True, 10, labels=train.labels),
            lr=0.01, batch_size=100, client_fraction=1.0, seed=10, eval_every=0)
fl.round()
fl.round()
torch.cuda.synchronize()
fl.sync_rounds = False
times.clear()
rt = []
for _ in range(5):
    t = time.perf_counter()
    fl.round()
    rt.append(time.perf_counter() - t)
t = time.perf_counter()
torch.cuda.synchronize()
print("graph_run host ms:", [round(1e3 * x, 2) for x in times])
print("round host ms:", [round(1e3 * x, 2) for x in rt], "final sync ms:", round(1e3 * (time.perf_counter() - t), 2))
