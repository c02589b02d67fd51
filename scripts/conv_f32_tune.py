"""Offline tuner of the fp32 conv launch plans (tile BP x BQ, split-K) for the ResNet-18 CIFAR layers.

For every conv geometry of ResNet-18 at the headline's client counts (G = 8, 4, 2, 1 clients of
batch 100) and every mode (FWD / DGRAD / WGRAD) it times each candidate plan with HIP events and
writes the best to ``ddl25spring_amd/ops/f32_plans.json`` (read by ``functional_f32.plan``), with
the achieved TF/s against the 157.3 TF/s fp32-MFMA peak.

    python scripts/conv_f32_tune.py --out gpurun_out/f32_plans.json [--groups 8 1]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

from ddl25spring_amd.ops import functional_f32 as F32  # noqa: E402
from ddl25spring_amd.ops.functional import ConvGeom  # noqa: E402

PEAK_TF = 157.3


def resnet18_geoms(G: int, N: int):
    gs = [ConvGeom(G, N, 32, 32, 32, 64, 1, 1, 1, 0)]  # im2col'd stem (1x1 on 32 channels)
    cin, hw = 64, 32
    for planes in (64, 128, 256, 512):
        stride = 1 if planes == 64 else 2
        ho = hw // stride
        gs.append(ConvGeom(G, N, hw, hw, cin, planes, 3, 3, stride, 1))
        gs.append(ConvGeom(G, N, ho, ho, planes, planes, 3, 3, 1, 1))
        if stride != 1:
            gs.append(ConvGeom(G, N, hw, hw, cin, planes, 1, 1, 2, 0))
        cin, hw = planes, ho
    return list(dict.fromkeys(gs))


def workspace_need(mode, g, bp, bq, split) -> int:
    import ctypes
    a = F32._args(g)
    a.split_k = split
    return int(F32._lib.kernels().ddl_convf32_workspace(ctypes.byref(a), mode, F32._cfg(F32.cfg_of(bp, bq))))


def resnet50_geoms(G: int, N: int):
    """ResNet-50 (ImageNet 224, torchvision v1.5 strides) conv geometries: im2col'd 7x7 stem (1x1 on
    160 channels) and the bottleneck 1x1 / 3x3 / strided convs."""
    gs = [ConvGeom(G, N, 112, 112, 160, 64, 1, 1, 1, 0)]
    cin, hw = 64, 56
    for planes, n in zip((64, 128, 256, 512), (3, 4, 6, 3)):
        for b in range(n):
            stride = 2 if (b == 0 and planes != 64) else 1
            ho = hw // stride
            gs.append(ConvGeom(G, N, hw, hw, cin, planes, 1, 1, 1, 0))
            gs.append(ConvGeom(G, N, hw, hw, planes, planes, 3, 3, stride, 1))
            gs.append(ConvGeom(G, N, ho, ho, planes, planes * 4, 1, 1, 1, 0))
            if b == 0:
                gs.append(ConvGeom(G, N, hw, hw, cin, planes * 4, 1, 1, stride, 0))
            cin, hw = planes * 4, ho
    return list(dict.fromkeys(gs))


LLM_SHAPES = ((288, 864), (288, 288), (288, 1536), (768, 288), (288, 32000))  # qkv, wo, w13, w2, LM head


def llama288_geoms(tokens=(8192, 2048)):
    """The LLaMA-288d linears as 1x1 convs over T token pixels (ops/llama_f32.LinearF32): T = 8192
    at pp=1 (batch 32 x 256), 2048 per micro-batch with a pipeline."""
    return [ConvGeom(1, T, 1, 1, C, K, 1, 1, 1, 0) for T in tokens for C, K in LLM_SHAPES]


def vendor_run(mode, g, x, w, dy, dw):
    """The same product on the vendor fp32 GEMM (torch.mm -> hipBLASLt), as LinearF32 runs it."""
    T = g.N * g.H * g.W
    x2, w2, d2, dw2 = x.view(T, g.C), w.view(g.K, g.C), dy.view(T, g.K), dw.view(g.K, g.C)
    return {F32.F_FWD: lambda: torch.mm(x2, w2.t()),
            F32.F_DGRAD: lambda: torch.mm(d2, w2),
            F32.F_WGRAD: lambda: dw2.addmm_(d2.t(), x2)}[mode]


EAGER = [False]


def timed(fn, reps):
    """Device time per call: ``reps`` calls captured in one graph and replayed (timing eager calls
    measured the host at one or two clients, where a launch's Python outlasts its kernels). With
    --eager-timing: eager calls, as the LLaMA linears' table was tuned (its whole graph-replayed
    step: eager-tuned 872k tok/s, graph-tuned 855k — per-launch differences within isolated-timing
    noise decided the choices, and the eager set won end to end)."""
    if EAGER[0]:
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps
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
    del g
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/f32_plans.json")
    ap.add_argument("--groups", type=int, nargs="*", default=[8, 1])
    ap.add_argument("--batch", type=int, default=100)
    ap.add_argument("--budget-s", type=float, default=240.0)
    ap.add_argument("--eager-timing", action="store_true", help="time eager calls (see timed)")
    ap.add_argument("--geoms-file", default="",
                    help="tune the (mode, geometry) launches a workload recorded (DDL_F32_RECORD=<file>)")
    ap.add_argument("--skip-halo", action="store_true",
                    help="skip launches the halo kernels take (FWD / DGRAD halo plans, halo WGRAD)")
    ap.add_argument("--math", default="mfma32", choices=list(F32.MATHS))
    ap.add_argument("--model", default="resnet18", choices=("resnet18", "resnet50", "llama288"))
    a = ap.parse_args()
    EAGER[0] = a.eager_timing
    F32.set_math(a.math)
    prefix = "" if a.math == "mfma32" else f"{a.math}:"
    engines = ("x6", "mfma32") if a.math == "auto" else (None,)
    dev = torch.device("cuda")
    F32.ensure_workspace(dev)
    t_start = time.time()
    plans, report = {}, []
    geoms = {"resnet50": resnet50_geoms, "resnet18": resnet18_geoms,
             "llama288": lambda G, N: llama288_geoms()}[a.model]
    only = None
    if a.geoms_file:  # recorded launches: their geometries, and per geometry only the recorded modes
        rec = json.loads(Path(a.geoms_file).read_text())
        only = {}
        for r in rec:
            only.setdefault(ConvGeom(*r["geom"]), set()).add(r["mode"])
        geoms = lambda G, N: list(only)  # noqa: E731
    for G in (a.groups if a.model != "llama288" and only is None else [1]):
        for g in geoms(G, a.batch):
            x = torch.randn(g.G, g.N, g.H, g.W, g.C, device=dev)
            w = torch.randn(g.G, g.K, g.R, g.S, g.C, device=dev) * 0.05
            dy = torch.randn(g.G, g.N, g.P, g.Q, g.K, device=dev)
            dw = torch.zeros_like(w)
            flops = 2 * g.G * g.N * g.P * g.Q * g.K * g.R * g.S * g.C
            for mode, name in ((F32.F_FWD, "fwd"), (F32.F_DGRAD, "dgrad"), (F32.F_WGRAD, "wgrad")):
                if only is not None and name not in only[g]:
                    continue
                if only is None and mode == F32.F_DGRAD and g.C in (32, 160) and g.R == 1:
                    continue  # the (im2col'd) stem needs no input gradient
                if a.skip_halo and (F32.uses_halo(mode, g) or (mode == F32.F_WGRAD and F32.uses_halo_wgrad(g))):
                    continue
                F32._OVERRIDE.pop((mode, g), None)
                F32._PLANS.pop((mode, g), None)
                heur = F32.plan(mode, g)
                run = {F32.F_FWD: lambda: F32.conv_fwd(x, w, g, stats=F32.SlotStats()),
                       F32.F_DGRAD: lambda: F32.conv_dgrad(dy, w, g),
                       F32.F_WGRAD: lambda: F32.conv_wgrad(dy, x, g, dw)}[mode]
                res = []
                for eng in engines:
                    for bp in (64, 128):
                        for bq in (64, 128):
                            Pd, Qd, _, nph = F32._dims(mode, g)
                            tiles = -(-Pd // bp) * -(-Qd // bq) * nph * g.G
                            for split in ((1, 2, 4, 8, 16, 32, 64, 128) if G <= 2 else (1, 2, 4, 8, 16, 32)):
                                if split > 1 and tiles * split > 8192:
                                    break  # the grid is already wide: deeper split-K only adds epilogue work
                                F32.set_plan(mode, g, bp, bq, split, eng)
                                if split > 1 and workspace_need(mode, g, bp, bq, split) > F32.WS_CAP:
                                    continue  # would silently run unsplit
                                try:
                                    ms = timed(run, 10)
                                except Exception as e:  # noqa: BLE001 (e.g. workspace too small)
                                    print("skip", name, g, bp, bq, split, e, flush=True)
                                    continue
                                res.append((ms, bp, bq, split, eng))
                F32._OVERRIDE.pop((mode, g), None)
                F32._PLANS.pop((mode, g), None)
                res.sort(key=lambda r: r[0])
                ms, bp, bq, split, eng = res[0]
                hcfg = heur[0] & ~F32.X6_BIT
                hms = next((r[0] for r in res if F32.cfg_of(r[1], r[2]) == hcfg and r[3] == heur[1]
                            and r[4] in (None, "x6")), None)
                key = f"{prefix}{name}:{g.G},{g.N},{g.H},{g.W},{g.C},{g.K},{g.R},{g.S},{g.stride},{g.pad}"
                plans[key] = [bp, bq, split] + ([eng] if eng else [])
                best_other = None
                if a.math == "auto":  # the other engine's best, for the report
                    best_other = next((round(r[0], 4) for r in res if r[4] != eng), None)
                row = dict(math=a.math, mode=name, G=g.G, N=g.N, H=g.H, C=g.C, K=g.K, R=g.R, stride=g.stride,
                           best_ms=round(ms, 4), plan=plans[key], other_engine_ms=best_other,
                           tflops=round(flops / ms / 1e9, 1),
                           pct_peak=round(100 * flops / ms / 1e9 / PEAK_TF, 1),
                           heuristic_ms=None if hms is None else round(hms, 4))
                if a.model == "llama288":  # plain GEMMs: the vendor fp32 GEMM is a candidate too
                    bms = timed(vendor_run(mode, g, x, w, dy, dw), 10)
                    row["vendor_ms"] = round(bms, 4)
                    if bms < 0.97 * ms:
                        plans["blas:" + key[len(prefix):]] = [round(bms, 4), round(ms, 4)]
                report.append(row)
                print(json.dumps(row), flush=True)
                if time.time() - t_start > a.budget_s:
                    break
            del x, w, dy, dw
            if time.time() - t_start > a.budget_s:
                print("budget reached", flush=True)
                break
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    Path(a.out).write_text(json.dumps({"plans": plans, "report": report}, indent=1))
    print("wrote", a.out)


if __name__ == "__main__":
    main()
