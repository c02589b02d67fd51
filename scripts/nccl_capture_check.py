"""Does HIP-graph capture coexist with a live RCCL process group (its watchdog thread polling
work events) on one GPU? Runs FedAvg rounds (round graph capture + tuner captures) with a
world-size-1 NCCL group carrying all-reduces between rounds, under the given capture mode.
    PYTHONPATH=. python scripts/nccl_capture_check.py thread_local|global"""
import sys

import torch
import torch.distributed as dist

mode = sys.argv[1] if len(sys.argv) > 1 else "thread_local"
dist.init_process_group("nccl", init_method="tcp://127.0.0.1:29811", rank=0, world_size=1)
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
import ddl25spring_amd.fl.local as L  # noqa: E402
import ddl25spring_amd.ops.autotune as AT  # noqa: E402
from ddl25spring_amd.data.images import DeviceImageDataset, synthetic_images  # noqa: E402
from ddl25spring_amd.data.split import split  # noqa: E402
from ddl25spring_amd.fl.algorithms import FedAvg  # noqa: E402
from ddl25spring_amd.models import resnet18_cifar  # noqa: E402
from ddl25spring_amd.runtime.dist import DistContext  # noqa: E402

L.CAPTURE_MODE = AT.CAPTURE_MODE = mode
x = torch.ones(1 << 22, device=dev)
arr = synthetic_images("cifar10", 2000, seed=0)
fa = FedAvg(resnet18_cifar, DeviceImageDataset(arr, dev), split(2, True, 0, labels=arr.labels), lr=0.01,
            batch_size=100, client_fraction=1.0, seed=0, ctx=DistContext(device=dev), eval_every=0)
for r in range(3):
    for _ in range(10):
        dist.all_reduce(x)  # in flight while the round starts (and, in round 0, captures)
    fa.round()
    torch.cuda.synchronize()
    print(f"mode={mode} round {r} ok", flush=True)
dist.destroy_process_group()
