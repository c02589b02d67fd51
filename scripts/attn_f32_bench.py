"""fp32 causal attention kernels alone (the LLaMA-288d shape: batch 32, ctx 256, 6 heads of 48):
forward + backward repeated, for PMC passes (scripts/gpu/pmc_attn.sh).

    python scripts/attn_f32_bench.py [--reps 20]
"""
from __future__ import annotations

import argparse
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from ddl25spring_amd.ops.llama_f32 import AttentionF32  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=32)
    ap.add_argument("--S", type=int, default=256)
    ap.add_argument("--H", type=int, default=6)
    ap.add_argument("--hd", type=int, default=48)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    qkv = torch.randn(a.B, a.S, 3 * a.H * a.hd, device="cuda", requires_grad=True)
    g = torch.randn(a.B, a.S, a.H * a.hd, device="cuda")
    for _ in range(a.reps):
        o = AttentionF32.apply(qkv, a.H, a.hd)
        o.backward(g)
    torch.cuda.synchronize()
    print("done", flush=True)


if __name__ == "__main__":
    main()
