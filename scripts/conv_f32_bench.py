"""One fp32 conv geometry, repeated launches — the target of PMC passes (scripts/gpu/pmc_f32.sh).

    python scripts/conv_f32_bench.py --math x6 --mode fwd --G 8 --layer c64 [--reps 20]
"""
from __future__ import annotations

import argparse
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from ddl25spring_amd.ops import functional_f32 as F32  # noqa: E402
from ddl25spring_amd.ops.functional import ConvGeom  # noqa: E402

LAYERS = {"c64": (32, 64, 64, 3, 1), "c128": (16, 128, 128, 3, 1), "c256": (8, 256, 256, 3, 1),
          "c512": (4, 512, 512, 3, 1), "c128s2": (32, 64, 128, 3, 2), "sc128": (32, 64, 128, 1, 2)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--math", default="x6", choices=list(F32.MATHS))
    ap.add_argument("--mode", default="fwd", choices=["fwd", "dgrad", "wgrad"])
    ap.add_argument("--G", type=int, default=8)
    ap.add_argument("--N", type=int, default=100)
    ap.add_argument("--layer", default="c64", choices=list(LAYERS))
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--halo", type=int, default=1, help="0: never the halo kernel (conv_x6h.hip)")
    ap.add_argument("--dybn", type=int, default=0, help="dgrad: dY operand = BN backward (dy_bn), 2: + write-out")
    ap.add_argument("--epi", default="", choices=["", "mbn", "rmb"],
                    help="dgrad epilogue of the network: mbn = producer BN reduce + recomputed ReLU mask "
                         "(a block's conv2), rmb = residual + mask tensor + BN reduce (a block's conv1)")
    ap.add_argument("--pin", default="", help="pin a plan: 'bp/bq/split[/x6h]' (x6h = the halo kernel)")
    a = ap.parse_args()
    F32.set_math(a.math)
    F32.set_halo(bool(a.halo))
    H, C, K, R, st = LAYERS[a.layer]
    g = ConvGeom(a.G, a.N, H, H, C, K, R, R, st, (R - 1) // 2)
    dev = torch.device("cuda")
    if a.pin:
        f = a.pin.replace(",", "/").split("/")
        mode_id = {"fwd": F32.F_FWD, "dgrad": F32.F_DGRAD, "wgrad": F32.F_WGRAD}[a.mode]
        F32.set_plan(mode_id, g, int(f[0]), int(f[1]), int(f[2]), *(f[3:4]))
    x = torch.randn(g.G, g.N, g.H, g.W, g.C, device=dev)
    w = torch.randn(g.G, g.K, g.R, g.S, g.C, device=dev) * 0.05
    dy = torch.randn(g.G, g.N, g.P, g.Q, g.K, device=dev)
    dw = torch.zeros_like(w)
    xb, coef = torch.randn_like(dy), torch.randn(g.G, 3, g.K, device=dev)
    dc = torch.empty_like(dy) if a.dybn == 2 else None
    dyb = dict(dy_bn=(xb, coef), dy_bn_out=dc) if a.dybn else {}
    if a.epi:
        bx = torch.randn(g.G, g.N, g.H, g.W, g.C, device=dev)
        mean, rstd = torch.randn(g.G, g.C, device=dev) * 0.1, torch.rand(g.G, g.C, device=dev) + 0.5
        dyb["bn"] = (bx, mean, rstd)
        if a.epi == "mbn":
            dyb["mask_bn"] = (torch.rand(g.G, g.C, device=dev) + 0.5, torch.randn(g.G, g.C, device=dev))
        else:
            dyb["residual"] = torch.randn(g.G, g.N, g.H, g.W, g.C, device=dev)
            dyb["mask"] = torch.randn(g.G, g.N, g.H, g.W, g.C, device=dev)
    run = {"fwd": lambda: F32.conv_fwd(x, w, g, stats=F32.SlotStats()),
           "dgrad": lambda: F32.conv_dgrad(dy, w, g, **dyb),
           "wgrad": lambda: F32.conv_wgrad(dy, x, g, dw)}[a.mode]
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        run()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.reps
    fl = 2 * g.G * g.N * g.P * g.Q * g.K * g.R * g.S * g.C
    mode = {"fwd": F32.F_FWD, "dgrad": F32.F_DGRAD, "wgrad": F32.F_WGRAD}[a.mode]
    print(f"{a.math} halo={a.halo} dybn={a.dybn} epi={a.epi or '-'} {a.mode} G={a.G} {a.layer}: {ms:.4f} ms {fl / ms / 1e9:.1f} TF/s "
          f"plan={F32.plan(mode, g)}")


if __name__ == "__main__":
    main()
