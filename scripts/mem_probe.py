"""Peak device memory of the graph-captured fp32 FedAvg round (bench.py's setup) per clients / overlap."""
import os, sys, time, torch
sys.path.insert(0, str(__import__("pathlib").Path(__file__).resolve().parent.parent))
from ddl25spring_amd.data.images import DeviceImageDataset, synthetic_images
from ddl25spring_amd.data.split import split
from ddl25spring_amd.fl.algorithms import FedAvg
from ddl25spring_amd.models import resnet18_cifar
C = int(sys.argv[1])
dev = torch.device("cuda")
train = synthetic_images("cifar10", 6250 * C, seed=0)
ds = DeviceImageDataset(train, dev)
fl = FedAvg(lambda groups: resnet18_cifar(10, groups=groups, precision="fp32"), ds, split(C, True, 10, labels=train.labels),
            lr=0.01, batch_size=100, local_epochs=1, client_fraction=1.0, seed=10, use_graph=True, eval_every=0)
torch.cuda.reset_peak_memory_stats()
for _ in range(2):
    fl.round()
torch.cuda.synchronize()
print(f"clients={C} overlap={os.environ.get('DDL_WGRAD_OVERLAP','auto')} peak_alloc={torch.cuda.max_memory_allocated()/2**30:.1f} GiB "
      f"reserved={torch.cuda.memory_reserved()/2**30:.1f} GiB", flush=True)
