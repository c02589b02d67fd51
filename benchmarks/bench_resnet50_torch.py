"""Reference-equivalent baseline for BASELINE config 3: stock PyTorch-ROCm ResNet-50 (torchvision v1.5
layout, ``models/torch_ref.py``) training in fp32 on one GPU — SGD momentum 0.9, wd 1e-4, synthetic
ImageNet-shaped batch, channels_last (MIOpen's default find; --benchmark for its exhaustive search). The number the
native fp32 path (``bench_resnet50_dp.py``) is compared against.

    python benchmarks/bench_resnet50_torch.py --batch 256 --steps 8 --warmup 3
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import torch
import torch.nn.functional as F

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from ddl25spring_amd.models.torch_ref import torch_resnet50_imagenet  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--benchmark", action="store_true", help="cudnn.benchmark (MIOpen exhaustive find: minutes)")
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = a.benchmark
    import threading

    def heartbeat():  # MIOpen's first-use kernel search / compilation runs for minutes without output
        t0 = time.time()
        while True:
            time.sleep(30)
            print(f"[heartbeat] {time.time() - t0:.0f} s", file=sys.stderr, flush=True)
    threading.Thread(target=heartbeat, daemon=True).start()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    m = torch_resnet50_imagenet(1000).to(dev).to(memory_format=torch.channels_last)
    opt = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    x = torch.randn(a.batch, 3, 224, 224, device=dev).to(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (a.batch,), device=dev)

    def step():
        opt.zero_grad(set_to_none=True)
        F.cross_entropy(m(x), y).backward()
        opt.step()
    for i in range(a.warmup):
        step()
        torch.cuda.synchronize()
        print(f"warmup step {i} done", file=sys.stderr, flush=True)  # MIOpen compiles kernels on first use
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(json.dumps({"metric": "ResNet-50 images/s (ImageNet-shape) [stock PyTorch fp32 reference-equivalent]",
                      "value": round(a.batch * a.steps / dt, 1), "unit": "images/s", "n_gpus": 1,
                      "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(1e3 * dt / a.steps, 3),
                      "dtype": "fp32", "data": "synthetic",
                      "config": {"model": "resnet50-imagenet", "global_batch": a.batch, "channels_last": True}}))


if __name__ == "__main__":
    main()
