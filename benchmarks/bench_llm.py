"""LLaMA (dmodel 288, 6 heads, 6 layers, ctx 256, 32k vocab — the tutorial_1b model) training
tokens/s over a DP x PP grid (world = dp * pp). Synthetic TinyStories-shaped token stream."""
from __future__ import annotations

import argparse

from _common import emit


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--dp", type=int, default=0, help="default: world // pp")
    ap.add_argument("--pp", type=int, default=1)
    ap.add_argument("--batch", type=int, default=32, help="per-pipeline batch")
    ap.add_argument("--micro", type=int, default=0,
                    help="micro-batches per pipeline (default: 4 with a pipeline, 1 without — at pp=1 "
                         "micro-batching is only gradient accumulation: same batch, 2.2x slower)")
    ap.add_argument("--schedule", default="1f1b")
    ap.add_argument("--precision", default="both", choices=("fp32", "bf16", "both"),
                    help="fp32 = the reference's precision (first line); bf16 = the bf16-MFMA path "
                         "(labelled second line); both (default) prints both")
    args = ap.parse_args()
    from ddl25spring_amd.apps.llm import LLMConfig, train_llm
    from ddl25spring_amd.runtime import dist as rdist
    ctx = rdist.init()
    dp = args.dp or ctx.world // args.pp
    if not args.micro:
        args.micro = 4 if args.pp > 1 else 1
    precs = ("fp32", "bf16") if args.precision == "both" else (args.precision,)
    for prec in precs:
        cfg = LLMConfig(dp=dp, pp=args.pp, batch_size=args.batch, micro_batches=args.micro,
                        schedule=args.schedule, iters=args.steps, log_every=10 ** 9, precision=prec)
        out = train_llm(cfg, ctx, log=None, warmup=args.warmup)
        emit(ctx, metric="LLaMA-288d training tokens/s" + ("" if prec == "fp32" else " (bf16 MFMA path)"),
             value=round(out["tokens_per_s"], 1),
             unit="tokens/s", n_gpus=ctx.world, steps=args.steps, warmup=args.warmup,
             ms_per_step=round(out["ms_per_iter"], 3), higher_is_better=True, scaling="weak",
             vs_baseline=None, dtype=prec, data="synthetic",
             config={"model": "llama-288d-6L", "global_batch": dp * args.batch, "seq_len": 256,
                     "parallelism": f"dp{dp}xpp{args.pp}", "micro_batches": args.micro,
                     "schedule": args.schedule})
    rdist.shutdown()


if __name__ == "__main__":
    main()
