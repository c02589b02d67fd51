"""Stride-1 1x1 convs ARE plain GEMMs (NHWC): per mode, the fp32 conv engine on its current plan
(tuned table / heuristic) vs the vendor true-fp32 GEMM (torch.mm -> hipBLASLt) on the same product.

    python scripts/gemm_vendor_probe.py --model resnet50 [--batch 256]
"""
from __future__ import annotations

import argparse
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
sys.path.insert(0, str(Path(__file__).resolve().parent))
from conv_f32_tune import llama288_geoms, resnet50_geoms, timed, vendor_run  # noqa: E402
from ddl25spring_amd.ops import functional_f32 as F32  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50", choices=("resnet50", "llama288"))
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda")
    geoms = resnet50_geoms(1, a.batch) if a.model == "resnet50" else llama288_geoms()
    tot_n = tot_b = 0.0
    for g in geoms:
        if g.R != 1 or g.stride != 1:
            continue
        x = torch.randn(g.G, g.N, g.H, g.W, g.C, device=dev)
        w = torch.randn(g.G, g.K, g.R, g.S, g.C, device=dev) * 0.05
        dy = torch.randn(g.G, g.N, g.P, g.Q, g.K, device=dev)
        dw = torch.zeros_like(w)
        fl = 2 * g.N * g.H * g.W * g.C * g.K
        line = []
        for mode, name in ((F32.F_FWD, "fwd"), (F32.F_DGRAD, "dgrad"), (F32.F_WGRAD, "wgrad")):
            nat = {F32.F_FWD: lambda: F32.conv_fwd(x, w, g, stats=F32.SlotStats()),
                   F32.F_DGRAD: lambda: F32.conv_dgrad(dy, w, g),
                   F32.F_WGRAD: lambda: F32.conv_wgrad(dy, x, g, dw)}[mode]
            n_ms = timed(nat, a.reps)
            b_ms = timed(vendor_run(mode, g, x, w, dy, dw), a.reps)
            tot_n += n_ms
            tot_b += min(n_ms, b_ms)
            line.append(f"{name} native {n_ms * 1e3:7.1f} us ({fl / n_ms / 1e9:5.1f} TF/s) vendor {b_ms * 1e3:7.1f} us "
                        f"({fl / b_ms / 1e9:5.1f})")
        print(f"{g.N}x{g.H}x{g.W} {g.C:4d}->{g.K:4d} | " + " | ".join(line), flush=True)
        del x, w, dy, dw
    print(f"sum native {tot_n:.2f} ms, best-of {tot_b:.2f} ms (each geometry once)")


if __name__ == "__main__":
    main()
