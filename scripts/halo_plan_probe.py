"""Halo-kernel plan sweep (BP x split-K) per ResNet-18 stride-1 3x3 layer and client count, in
one process: device time of FWD (with BN statistics) and DGRAD per pinned plan, against the
default plan (functional_f32._halo_plan).

    python scripts/halo_plan_probe.py [--G 1 2 4 8] [--reps 20] [--out gpurun_out/x6h_plans.json]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
sys.path.insert(0, str(Path(__file__).resolve().parent))
from ddl25spring_amd.ops import functional_f32 as F32  # noqa: E402
from ddl25spring_amd.ops.functional import ConvGeom  # noqa: E402

def timed(fn, reps):
    """Device time per call: reps calls captured in one graph (the eager calls are host-bound at
    one or two clients), replayed after a warm-up."""
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


LAYERS = {"c64": (32, 64), "c128": (16, 128), "c256": (8, 256), "c512": (4, 512)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--G", type=int, nargs="*", default=[1])
    ap.add_argument("--N", type=int, default=100)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--model", default="resnet18", choices=("resnet18", "resnet50", "resnet50_flat1x1"))
    ap.add_argument("--out", default="", help="write the best plans as 'x6h:' table entries (scripts/merge_plans.py)")
    a = ap.parse_args()
    plans, report = {}, []
    dev = torch.device("cuda")
    F32.ensure_workspace(dev)
    for G in a.G:
        if a.model == "resnet50":  # the bottleneck 3x3 stride-1 convs (rows padded to a power of two)
            from conv_f32_tune import resnet50_geoms
            layers = [(f"r50_{g.H}x{g.C}", g) for g in resnet50_geoms(G, a.N) if g.R == 3 and g.stride == 1]
        elif a.model == "resnet50_flat1x1":  # stride-1 1x1 convs as rows of 128 pixels (FLAT1X1 FWD / DGRAD)
            from conv_f32_tune import resnet50_geoms
            flat = [F32._launch_geom(g, "f") for g in resnet50_geoms(G, a.N) if g.R == 1 and g.stride == 1]
            layers = [(f"r50_1x1_{g.C}to{g.K}_{g.H}rows", g) for g in dict.fromkeys(flat) if g.W == 128]
        else:
            layers = [(name, ConvGeom(G, a.N, H, H, C, C, 3, 3, 1, 1)) for name, (H, C) in LAYERS.items()]
        for name, g in layers:
            C = g.C
            x = torch.randn(g.G, g.N, g.H, g.W, g.C, device=dev)
            w = torch.randn(g.G, g.K, g.R, g.S, g.C, device=dev) * 0.05
            dy = torch.randn(g.G, g.N, g.P, g.Q, g.K, device=dev)
            for mode, mname in ((F32.F_FWD, "fwd"), (F32.F_DGRAD, "dgrad")):
                run = (lambda: F32.conv_fwd(x, w, g, stats=F32.SlotStats())) if mode == F32.F_FWD else \
                    (lambda: F32.conv_dgrad(dy, w, g))
                F32.clear_plan(mode, g)
                dflt = F32.plan(mode, g)
                t0 = timed(run, a.reps)
                res = []
                for bp in (64, 128):
                    for split in (1, 2, 4, 8):
                        if C // 16 < split * 4:
                            continue
                        F32.set_plan(mode, g, bp, 128, split, "x6h")
                        try:
                            res.append((timed(run, a.reps), bp, split))
                        except Exception as e:  # noqa: BLE001
                            print("skip", name, mname, bp, split, e, flush=True)
                F32.clear_plan(mode, g)
                if not res:
                    continue
                res.sort()
                best = res[0]
                key = f"x6h:{mname}:{g.G},{g.N},{g.H},{g.W},{g.C},{g.K},{g.R},{g.S},{g.stride},{g.pad}"
                plans[key] = [best[1], 128, best[2]]
                report.append(dict(G=G, layer=name, mode=mname, default=list(dflt), default_us=round(t0 * 1e3, 1),
                                   best=plans[key], best_us=round(best[0] * 1e3, 1)))
                print(f"G={G} {name} {mname}: default {dflt} {t0 * 1e3:6.1f} us | best bp={best[1]} split={best[2]} "
                      f"{best[0] * 1e3:6.1f} us | " + " ".join(f"{b}/{s}:{t * 1e3:.1f}" for t, b, s in res), flush=True)
            if a.model != "resnet50_flat1x1" and F32.uses_halo_wgrad(g):  # halo WGRAD: slice count sweep
                dw = torch.zeros_like(w)
                base = (g.K // 64) * (g.C // 32) * G
                t0 = timed(lambda: F32.conv_wgrad(dy, x, g, dw), a.reps)
                res = []
                for split in (1, 2, 4, 8, 16, 32, 64, 128):
                    if base * split > 2048:
                        break
                    res.append((timed(lambda: F32.conv_wgrad(dy, x, g, dw, split_k=split), a.reps), split))
                res.sort()
                key = f"x6hw:wgrad:{g.G},{g.N},{g.H},{g.W},{g.C},{g.K},{g.R},{g.S},{g.stride},{g.pad}"
                plans[key] = [res[0][1]]
                report.append(dict(G=G, layer=name, mode="wgrad", default_us=round(t0 * 1e3, 1),
                                   best=plans[key], best_us=round(res[0][0] * 1e3, 1)))
                print(f"G={G} {name} wgrad(x6hw): default {t0 * 1e3:6.1f} us | best split={res[0][1]} "
                      f"{res[0][0] * 1e3:6.1f} us | " + " ".join(f"{s_}:{t * 1e3:.1f}" for t, s_ in res), flush=True)
                del dw
            del x, w, dy
    if a.out:
        Path(a.out).parent.mkdir(parents=True, exist_ok=True)
        Path(a.out).write_text(json.dumps({"plans": plans, "report": report}, indent=1))


if __name__ == "__main__":
    main()
