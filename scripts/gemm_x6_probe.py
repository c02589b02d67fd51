"""Timing probes of the X6 GEMM (gemm_x6.hip GemmX6Args.probe; results wrong by design): which of
DMA staging, fragment reads and MFMAs bounds a shape. python scripts/gemm_x6_probe.py"""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from ddl25spring_amd.ops import gemm_x6 as G  # noqa: E402
from gemm_x6_bench import timeit  # noqa: E402

dev = torch.device("cuda")
T = 8192
cases = [("head_fwd", 32000, 288, False, False), ("qkv_wgrad1", 864, 8192, True, True),
         ("w13_fwd", 1536, 288, False, False)]
for name, P, K, amn, bmn in cases:
    a = torch.randn(K, P, device=dev) if amn else torch.randn(P, K, device=dev)
    b = torch.randn(K, T if name != "qkv_wgrad1" else 288, device=dev) if bmn else torch.randn(T, K, device=dev)
    pa, pb = G.split(a), G.split(b)
    N = b.shape[1] if bmn else b.shape[0]
    out = torch.empty(N, P, device=dev)
    for plan in ([4, 4, 3, 1], [3, 4, 3, 1], [4, 2, 4, 1]):
        for probe in (0, 1, 2, 4, 8, 6, 3, 15):
            G._PLANS.clear()
            G._PLANS[(P, N, K)] = tuple(plan)
            G.PROBE[0] = probe
            us = timeit(lambda: G.gemm(pa, amn, pb, bmn, out), iters=10)
            print(json.dumps({"case": name, "plan": plan, "probe": probe, "us": round(us, 1),
                              "tflops": round(2 * P * N * K / us / 1e6, 1)}), flush=True)
G.PROBE[0] = 0
