"""Empty-loop cost of the X6 GEMM skeleton vs reduction length (probe 15 / 16)."""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from ddl25spring_amd.ops import gemm_x6 as G  # noqa: E402
from gemm_x6_bench import timeit  # noqa: E402

dev = torch.device("cuda")
for K in (1024, 4096, 8192):
    for P, N in ((256, 128), (2048, 2048)):
        a = torch.randn(K, P, device=dev)
        b = torch.randn(K, N, device=dev)
        pa, pb = G.split(a), G.split(b)
        out = torch.empty(N, P, device=dev)
        for plan in ((4, 4, 3, 1), (4, 2, 4, 1)):
            for probe in (16, 15, 0):
                G._PLANS.clear()
                G._PLANS[(P, N, K)] = plan
                G.PROBE[0] = probe
                us = timeit(lambda: G.gemm(pa, True, pb, True, out), iters=5)
                print(json.dumps({"K": K, "P": P, "N": N, "plan": plan, "probe": probe, "us": round(us, 1),
                                  "tflops": round(2 * P * N * K / us / 1e6, 1)}), flush=True)
