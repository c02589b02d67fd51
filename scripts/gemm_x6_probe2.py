"""Kernel-trace companion of gemm_x6_probe.py: one launch per (case, probe), for rocprofv3."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from ddl25spring_amd.ops import gemm_x6 as G  # noqa: E402

dev = torch.device("cuda")
cases = [("head_fwd", 32000, 288, 8192, False, False), ("qkv_wgrad1", 864, 8192, 288, True, True)]
for name, P, K, N, amn, bmn in cases:
    a = torch.randn(K, P, device=dev) if amn else torch.randn(P, K, device=dev)
    b = torch.randn(K, N, device=dev) if bmn else torch.randn(N, K, device=dev)
    pa, pb = G.split(a), G.split(b)
    out = torch.empty(N, P, device=dev)
    G._PLANS.clear()
    G._PLANS[(P, N, K)] = (4, 4, 3, 1)
    for probe in (0, 16, 15, 7, 8, 1):
        G.PROBE[0] = probe
        for _ in range(3):
            G.gemm(pa, amn, pb, bmn, out)
        torch.cuda.synchronize()
        print(name, probe, flush=True)
