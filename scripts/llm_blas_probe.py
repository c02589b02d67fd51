"""Vendor fp32 GEMM (torch.mm -> hipBLASLt / rocBLAS) on the LLaMA-288d linear shapes, per mode, for
comparison with the fp32 conv engine (scripts/llm_linear_bench.py): device time, TF/s, and the
max relative error against a float64 product.

    python scripts/llm_blas_probe.py [--tf32 0|1]
"""
from __future__ import annotations

import argparse

import torch

SHAPES = {"qkv": (288, 864), "wo": (288, 288), "w13": (288, 1536), "w2": (768, 288), "head": (288, 32000)}


def timed(fn, reps):
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=8192)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--tf32", type=int, default=0)
    a = ap.parse_args()
    torch.backends.cuda.matmul.allow_tf32 = bool(a.tf32)
    dev = torch.device("cuda")
    T = a.T
    for name, (C, K) in SHAPES.items():
        x = torch.randn(T, C, device=dev)
        w = torch.randn(K, C, device=dev) * 0.05
        dy = torch.randn(T, K, device=dev)
        ops = {"fwd": (lambda: x @ w.t(), lambda: x.double() @ w.double().t()),
               "dgrad": (lambda: dy @ w, lambda: dy.double() @ w.double()),
               "wgrad": (lambda: dy.t() @ x, lambda: dy.double().t() @ x.double())}
        line = []
        for mode, (f, ref) in ops.items():
            ms = timed(f, a.reps)
            r = ref()
            err = ((f().double() - r).abs().max() / r.abs().max()).item()
            line.append(f"{mode} {ms * 1e3:7.1f} us {2 * T * C * K / ms / 1e9:6.1f} TF/s err {err:.1e}")
        print(f"{name:5s} {C:4d}->{K:5d} tf32={a.tf32} | " + " | ".join(line), flush=True)


if __name__ == "__main__":
    main()
