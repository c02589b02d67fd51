"""Kernel nodes per captured local step of the 1-client ResNet-18 round graph (fl/local.py): capture
rounds chunked at 1 and 2 steps and count each graph's nodes with hipGraphGetNodes, so the
round-graph step limit (GRAPH_MAX_STEPS) can be stated in nodes.

    python scripts/graph_nodes.py
"""
from __future__ import annotations

import ctypes
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def nodes(g) -> int:
    hip = ctypes.CDLL("libamdhip64.so")
    n = ctypes.c_size_t(0)
    rc = hip.hipGraphGetNodes(ctypes.c_void_p(g.raw_cuda_graph()), None, ctypes.byref(n))
    assert rc == 0, rc
    return n.value


def main():
    import os
    os.environ["DDL_GRAPH_KEEP"] = "1"
    import ddl25spring_amd.fl.local as L
    from ddl25spring_amd.data.images import DeviceImageDataset, synthetic_images
    from ddl25spring_amd.data.split import split
    from ddl25spring_amd.fl.algorithms import FedAvg
    from ddl25spring_amd.models import resnet18_cifar
    from ddl25spring_amd.runtime.dist import DistContext
    dev = torch.device("cuda")
    out = {}
    for chunk in (1, 2, 4):
        L.GRAPH_MAX_STEPS = chunk
        arr = synthetic_images("cifar10", 100 * (chunk + 1), seed=0)  # chunk full steps + 1 full-size chunk
        fa = FedAvg(lambda groups: resnet18_cifar(10, groups=groups, precision="fp32"), DeviceImageDataset(arr, dev),
                    split(1, True, 10, labels=arr.labels), lr=0.05, batch_size=100, client_fraction=1.0, seed=1,
                    ctx=DistContext(device=dev), eval_every=0, use_graph=True)
        fa.round()
        torch.cuda.synchronize()
        counts = {str(k[2]): nodes(ents[0]["graph"]) for k, ents in fa.trainer._graphs.items()}
        out[chunk] = counts
    print(json.dumps({"graph_nodes_by_steps": out}))


if __name__ == "__main__":
    main()
