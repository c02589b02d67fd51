import sys, time
sys.path.insert(0, "benchmarks"); sys.path.insert(0, ".")
import torch
from ddl25spring_amd.data.images import DeviceImageDataset, load_images
from ddl25spring_amd.data.split import split
from ddl25spring_amd.fl.algorithms import FedAvg
from ddl25spring_amd.fl.attacks import make_attack
from ddl25spring_amd.models import resnet18_cifar
from ddl25spring_amd.runtime import dist as rdist
import bench_byzantine as BB
ctx = rdist.init()
train = load_images("cifar10", True, 50000)
parts = split(8, True, 0, labels=train.labels)
data = DeviceImageDataset(train, ctx.device)
for flip in (False, True):
    attack = make_attack("sign_flip", [2, 3])
    fa = FedAvg(resnet18_cifar, data, parts, lr=0.01, batch_size=100, client_fraction=1.0, seed=0,
                aggregator="mean", attack=attack, ctx=ctx, eval_every=0)
    if flip:
        fa.attack = BB._Both(attack, make_attack("label_flip", [0, 1]))
    for r in range(4):
        torch.cuda.synchronize(); t0 = time.perf_counter()
        fa.round()
        torch.cuda.synchronize()
        print(f"flip={flip} round {r}: {1e3*(time.perf_counter()-t0):.1f} ms graphs={list(fa.trainer._graphs.keys())} use_graph={fa.trainer.use_graph}", flush=True)
