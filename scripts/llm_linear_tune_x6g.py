"""Per-layer engine choice for the fp32 LLaMA linears between the two NATIVE engines: the X6 planes
GEMM (gemm_x6.hip; its operands split once per step) and the X6 / exact-fp32 conv engine
(conv_f32.hip, 1x1 conv over T "pixels", reading fp32 directly). For every linear of the
tutorial LLaMA (T = 8192 tokens) it times each product on both engines (the planes GEMM over a few
tile / split plans) and the plane splits each product needs, then picks per layer the combination
of the 2^3 engine assignments with the least total time (a split shared by two planes-GEMM products
is paid once). Writes 'lin:' (engine) and 'x6g:' (GEMM plan) entries into ops/f32_plans.json
(--write) and prints the table.

    python scripts/llm_linear_tune_x6g.py [--T 8192] [--write]
"""
from __future__ import annotations

import argparse
import itertools
import json
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from ddl25spring_amd.ops import functional as Fn  # noqa: E402
from ddl25spring_amd.ops import functional_f32 as F32  # noqa: E402
from ddl25spring_amd.ops import gemm_x6 as G  # noqa: E402

PLANS = [(4, 4, 3, 1), (3, 4, 3, 1), (4, 2, 4, 1), (3, 2, 4, 1), (2, 4, 4, 1), (4, 4, 3, 2), (3, 4, 3, 2),
         (3, 4, 3, 4), (4, 4, 3, 4), (3, 4, 3, 8), (4, 4, 3, 8), (3, 4, 3, 16), (4, 4, 3, 16), (3, 4, 3, 32)]


def timeit(fn, iters=10, warm=3):
    for _ in range(warm):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=8192)
    ap.add_argument("--write", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    T = args.T
    layers = [("qkv", 288, 864), ("wo", 288, 288), ("w13", 288, 1536), ("w2", 768, 288), ("head", 288, 32000)]
    entries = {}
    for name, C, K in layers:
        x = torch.randn(T, C, device=dev)
        w = torch.randn(K, C, device=dev) * 0.05
        dy = torch.randn(T, K, device=dev) * 0.01
        px, pw, pd = G.split(x), G.split(w), G.split(dy)
        t_split = {"x": timeit(lambda: G.split(x, px.data)), "w": timeit(lambda: G.split(w, pw.data)),
                   "dy": timeit(lambda: G.split(dy, pd.data))}
        geom = Fn.ConvGeom(1, T, 1, 1, C, K, 1, 1, 1, 0)
        x5, w5, d5 = x.view(1, T, 1, 1, C), w.view(1, K, 1, 1, C), dy.view(1, T, 1, 1, K)
        dwt = torch.zeros(1, K, 1, 1, C, device=dev)
        conv = {"fwd": timeit(lambda: Fn.conv_fwd(x5, w5, geom)),
                "dgrad": timeit(lambda: Fn.conv_dgrad(d5, w5, geom)),
                "wgrad": timeit(lambda: Fn.conv_wgrad(d5, x5, geom, dwt))}
        gemm_args = {"fwd": (pw, False, px, False, (T, K)), "dgrad": (pw, True, pd, False, (T, C)),
                     "wgrad": (px, True, pd, True, (K, C))}
        x6g, x6g_plan = {}, {}
        for mode, (pa, amn, pb, bmn, oshape) in gemm_args.items():
            out = torch.zeros(*oshape, device=dev)
            M, N = oshape[1], oshape[0]
            Kr = {"fwd": C, "dgrad": K, "wgrad": T}[mode]
            best = None
            for pl in PLANS:
                tiles = -(-M // (32 * pl[0])) * -(-N // (32 * pl[1]))
                if pl[3] > 1 and (Kr // 32) < pl[3] * 4:
                    continue
                if pl[3] > 1 and tiles >= 512:
                    continue
                G._PLANS.clear()
                G._PLANS[(M, N, Kr)] = pl
                t = timeit(lambda: G.gemm(pa, amn, pb, bmn, out, accumulate=mode == "wgrad"))
                if best is None or t < best[0]:
                    best = (t, pl)
            G._PLANS.clear()
            x6g[mode], x6g_plan[mode] = best
        # per layer: the engine assignment with the least total time (splits shared)
        choice = None
        for combo in itertools.product(("x6g", "conv"), repeat=3):
            eng = dict(zip(("fwd", "dgrad", "wgrad"), combo))
            t = sum(x6g[m] if eng[m] == "x6g" else conv[m] for m in eng)
            need = set()
            if "x6g" in (eng["fwd"], eng["wgrad"]):
                need.add("x")
            if "x6g" in (eng["fwd"], eng["dgrad"]):
                need.add("w")
            if "x6g" in (eng["dgrad"], eng["wgrad"]):
                need.add("dy")
            t += sum(t_split[k] for k in need)
            if choice is None or t < choice[0]:
                choice = (t, eng)
        rec = {"layer": name, "C": C, "K": K, "conv_us": {k: round(v, 1) for k, v in conv.items()},
               "x6g_us": {k: round(v, 1) for k, v in x6g.items()}, "x6g_plan": x6g_plan,
               "split_us": {k: round(v, 1) for k, v in t_split.items()}, "choice": choice[1],
               "total_us": round(choice[0], 1)}
        print(json.dumps(rec), flush=True)
        for m, e in choice[1].items():
            entries[f"lin:{m}:{T},{C},{K}"] = e
            M, N, Kr = {"fwd": (K, T, C), "dgrad": (C, T, K), "wgrad": (C, K, T)}[m]
            entries[f"x6g:{M},{N},{Kr}"] = list(x6g_plan[m])
    if args.write:
        path = ROOT / "ddl25spring_amd" / "ops" / "f32_plans.json"
        doc = json.loads(path.read_text())
        plans = doc.setdefault("plans", {})
        for k in [k for k in plans if k.startswith("blas:")]:
            del plans[k]  # the vendor GEMM is no longer a tuned choice
        plans.update(entries)
        path.write_text(json.dumps(doc, indent=1, sort_keys=True))
        print(f"wrote {len(entries)} entries to {path}")


if __name__ == "__main__":
    main()
