"""Per-layer conv kernel timing (fwd / dgrad / wgrad) for the client-batched ResNet-18 shapes,
optionally sweeping tile configs and comparing against PyTorch/MIOpen on the same shapes.

    python scripts/conv_bench.py [--sweep] [--miopen] [--G 8 --N 100]
Timing: HIP events around a captured graph of R back-to-back launches, median of 5 replays,
random bf16 data.
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from ddl25spring_amd.ops import functional as Fn  # noqa: E402
from ddl25spring_amd.ops.functional import ConvGeom  # noqa: E402


def resnet18_shapes(G, N):
    out = [("stem", ConvGeom(G, N, 32, 32, 32, 64, 1, 1, 1, 0))]
    spec = [(64, 32, 1), (128, 16, 2), (256, 8, 2), (512, 4, 2)]
    cin, h = 64, 32
    for planes, hw, stride in spec:
        if stride == 2:
            out.append((f"c{planes}s2", ConvGeom(G, N, h, h, cin, planes, 3, 3, 2, 1)))
            out.append((f"sc{planes}", ConvGeom(G, N, h, h, cin, planes, 1, 1, 2, 0)))
        out.append((f"c{planes}", ConvGeom(G, N, hw, hw, planes, planes, 3, 3, 1, 1)))
        cin, h = planes, hw
    return out


def timeit(fn, reps=10, rounds=5):
    """Median per-call time of `reps` calls replayed from one captured HIP graph (so small-grid
    kernels are not timed against Python/ctypes launch overhead, as in graph-captured training)."""
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        for _ in range(reps):
            fn()
    graph.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(rounds):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        graph.replay()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) / reps)
    return statistics.median(ts)


CFGS = Fn.CONV_TILES


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--G", type=int, default=8)
    ap.add_argument("--N", type=int, default=100)
    ap.add_argument("--sweep", action="store_true")
    ap.add_argument("--miopen", action="store_true")
    ap.add_argument("--json", default=None)
    ap.add_argument("--layers", default="", help="comma list of layer names to run (default all)")
    ap.add_argument("--splits", default="", help="FWD/DGRAD split-K counts to time, e.g. 1,2,4")
    ap.add_argument("--split-sweep", action="store_true", help="also sweep tiles x splits")
    ap.add_argument("--wh-splits", default="", help="halo WGRAD split-K counts to time, e.g. 4,8,16")
    ap.add_argument("--epi", action="store_true",
                    help="time with the fused epilogues of training (residual; mask + BN-backward reduce)")
    args = ap.parse_args()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    results = []
    tot = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0, "miopen": 0.0}
    for name, g in resnet18_shapes(args.G, args.N):
        if args.layers and name not in args.layers.split(","):
            continue
        x = torch.randn(g.G, g.N, g.H, g.W, g.C, device=dev).to(torch.bfloat16)
        w = (torch.randn(g.G, g.K, g.R, g.S, g.C, device=dev) * 0.05).to(torch.bfloat16)
        dy = torch.randn(g.G, g.N, g.P, g.Q, g.K, device=dev).to(torch.bfloat16)
        dw = torch.zeros(g.G, g.K, g.R, g.S, g.C, device=dev)
        st = Fn.stats_buffer(g.G, g.K, dev)  # fwd runs with the BN-statistics epilogue, as in training
        fl = g.flops()
        row = {"layer": name, "geom": str(g), "gflop": fl / 1e9}
        if args.epi:  # the training step's fused epilogues: fwd + residual, dgrad + mask + BN reduce
            res = torch.randn(g.G, g.N, g.P, g.Q, g.K, device=dev).to(torch.bfloat16)
            msk = torch.randn(g.G, g.N, g.H, g.W, g.C, device=dev).to(torch.bfloat16)
            mean = torch.zeros(g.G, g.C, device=dev)
            rstd = torch.ones(g.G, g.C, device=dev)
        modes = {
            "fwd": (lambda cfg, sk=0: Fn.conv_fwd(x, w, g, cfg=cfg, stats=st, split_k=sk, residual=res))
            if args.epi else (lambda cfg, sk=0: Fn.conv_fwd(x, w, g, cfg=cfg, stats=st, split_k=sk)),
            "dgrad": (lambda cfg, sk=0: Fn.conv_dgrad(dy, w, g, cfg=cfg, split_k=sk, mask=msk, bn=(x, mean, rstd)))
            if args.epi else (lambda cfg, sk=0: Fn.conv_dgrad(dy, w, g, cfg=cfg, split_k=sk)),
            "wgrad": lambda cfg: Fn.conv_wgrad(dy, x, g, dw, cfg=cfg),
        }
        for mode, f in modes.items():
            if mode == "dgrad" and name == "stem":
                continue
            t = timeit(lambda: f(0))
            row[mode] = {"ms": t, "tflops": fl / t / 1e9}
            tot[mode] += t
            if args.wh_splits and mode == "wgrad":
                row[mode]["halo_splits_us"] = {}
                for ns in (4, 5, 6):
                    hcfg = Fn.conv_cfg(64, 288, 32, ns, halo=True)
                    for k in args.wh_splits.split(","):
                        try:
                            row[mode]["halo_splits_us"][f"s{ns}/{k}"] = round(1e3 * timeit(
                                lambda: Fn.conv_wgrad(dy, x, g, dw, cfg=hcfg, splits=int(k))), 1)
                        except Exception:
                            pass
            if args.splits and mode != "wgrad":
                row[mode]["splits_us"] = {int(k): round(1e3 * timeit(lambda: f(0, int(k))), 1)
                                          for k in args.splits.split(",")}
                if args.split_sweep:  # (tile x split) grid: best combination
                    best = (1e9, None)
                    for bp, bq, bk, ns in [(128, 128, 64, 2), (128, 128, 32, 3), (64, 128, 64, 3),
                                           (128, 64, 64, 3), (64, 64, 64, 3), (128, 256, 32, 2),
                                           (256, 128, 32, 2)]:
                        if (g.C if mode == "fwd" else g.K) % bk:
                            continue
                        for k in [int(v) for v in args.splits.split(",")]:
                            tc = timeit(lambda: f(Fn.conv_cfg(bp, bq, bk, ns), k), reps=5, rounds=3)
                            if tc < best[0]:
                                best = (tc, f"{bp}x{bq}x{bk}s{ns}/k{k}")
                    row[mode]["splits_us"]["best"] = f"{best[0] * 1e3:.1f}@{best[1]}"
            if args.sweep:
                best = (t, 0)
                cands = [(f"{bp}x{bq}x{bk}s{ns}", Fn.conv_cfg(bp, bq, bk, ns))
                         for bp, bq, bk, ns in CFGS
                         if not ((mode == "fwd" and g.C % bk) or (mode == "dgrad" and g.K % bk))]
                if mode != "wgrad":  # halo-staged 3x3 stride-1 kernels (raise where ineligible)
                    cands += [(f"halo{bp}x{bq}s{ns}", Fn.conv_cfg(bp, bq, 32, ns, halo=True))
                              for bp, bq, ns in Fn.HALO_TILES]
                else:
                    cands.append(("halo64x288s4", Fn.conv_cfg(64, 288, 32, 4, halo=True)))
                for label, cfg in cands:
                    try:
                        tc = timeit(lambda: f(cfg), reps=5, rounds=3)
                    except Exception:
                        continue
                    row.setdefault(mode + "_sweep", {})[label] = round(fl / tc / 1e9, 1)
                    if tc < best[0]:
                        best = (tc, cfg)
                row[mode]["best_cfg"] = best[1]
                row[mode]["best_tflops"] = fl / best[0] / 1e9
        if args.miopen:
            xc = x[0].permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
            wc = w[0].permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)

            def mi():
                for _ in range(g.G):
                    torch.nn.functional.conv2d(xc, wc, None, g.stride, g.pad)
            t = timeit(mi)
            row["miopen_fwd"] = {"ms": t, "tflops": fl / t / 1e9}
            tot["miopen"] += t
        results.append(row)
        msg = f"{name:8s} {fl / 1e9:7.1f} GF"
        for mode in ("fwd", "dgrad", "wgrad"):
            if mode in row:
                msg += f" | {mode} {row[mode]['ms'] * 1e3:7.1f}us {row[mode]['tflops']:6.0f}TF"
                if "halo_splits_us" in row[mode]:
                    msg += f" halo-splits{row[mode]['halo_splits_us']}"
                if "splits_us" in row[mode]:
                    msg += f" split{row[mode]['splits_us']}"
                if "best_cfg" in row[mode]:
                    msg += f" (best {row[mode]['best_tflops']:.0f} @{row[mode]['best_cfg']:#x})"
                if mode + "_sweep" in row:
                    halo = {k: v for k, v in row[mode + "_sweep"].items() if k.startswith("halo")}
                    if halo:
                        msg += f" halo{halo}"
        if "miopen_fwd" in row:
            msg += f" | miopen fwd {row['miopen_fwd']['tflops']:6.0f}TF"
        print(msg, flush=True)
    print("totals (ms, one instance of each layer):", {k: round(v, 3) for k, v in tot.items()})
    if args.json:
        Path(args.json).write_text(json.dumps(results, indent=1))


if __name__ == "__main__":
    main()
