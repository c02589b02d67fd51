"""Probe matrix (gemm_x6.hip GemmX6Args.probe) on a large square-ish X6 GEMM and the LM-head FWD."""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from ddl25spring_amd.ops import gemm_x6 as G  # noqa: E402
from gemm_x6_bench import timeit  # noqa: E402

dev = torch.device("cuda")
cases = [("sq2048_k8192_mnmn", 2048, 2048, 8192, True, True), ("sq2048_k8192_kk", 2048, 2048, 8192, False, False),
         ("head_fwd", 32000, 8192, 288, False, False)]
for name, P, N, K, amn, bmn in cases:
    a = torch.randn(K, P, device=dev) if amn else torch.randn(P, K, device=dev)
    b = torch.randn(K, N, device=dev) if bmn else torch.randn(N, K, device=dev)
    pa, pb = G.split(a), G.split(b)
    out = torch.empty(N, P, device=dev)
    for plan in ((4, 4, 3, 1),):
        for probe in (0, 8):
            G._PLANS.clear()
            G._PLANS[(P, N, K)] = plan
            G.PROBE[0] = probe
            us = timeit(lambda: G.gemm(pa, amn, pb, bmn, out), iters=5)
            print(json.dumps({"case": name, "plan": plan, "probe": probe, "us": round(us, 1),
                              "tflops": round(2 * P * N * K / us / 1e6, 1)}), flush=True)
G.PROBE[0] = 0
