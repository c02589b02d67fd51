"""Command-line entry point: ``python -m ddl25spring_amd <program> [--field value ...]``.

Programs: fl (horizontal FL), vfl (centralized / split-NN / VAE / VFL-VAE on heart-disease),
gan (federated DCGAN), llm (LLaMA DP x PP). Every dataclass field of the program's config is a
flag (``--client-fraction 0.1``, ``--iid false``). Multi-rank: start under
``python -m ddl25spring_amd.runtime.launch -n W`` or torchrun (env rendezvous on 127.0.0.1);
rank r uses GPU r, RCCL between GPUs, gloo on CPU.
"""
from __future__ import annotations

import argparse
import dataclasses
import json
import sys
import typing


def _parse_bool(v: str) -> bool:
    if v.lower() in ("1", "true", "yes", "y", "on"):
        return True
    if v.lower() in ("0", "false", "no", "n", "off"):
        return False
    raise argparse.ArgumentTypeError(f"not a boolean: {v}")


def _add_fields(p: argparse.ArgumentParser, cls):
    hints = typing.get_type_hints(cls)
    for f in dataclasses.fields(cls):
        t = hints[f.name]
        base = [a for a in typing.get_args(t) if a is not type(None)]
        t = base[0] if base else t
        conv = _parse_bool if t is bool else t
        p.add_argument("--" + f.name.replace("_", "-"), dest=f.name, type=conv, default=f.default)


PROGRAMS = {
    "fl": ("apps.fl", "FLConfig", "run_fl"),
    "vfl": ("apps.vfl", "VFLConfig", "run_vfl"),
    "gan": ("apps.gan", "GANConfig", "run_gan"),
    "llm": ("apps.llm", "LLMConfig", "train_llm"),
}


def main(argv=None) -> int:
    import importlib
    ap = argparse.ArgumentParser(prog="python -m ddl25spring_amd", description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--device", default=None, help="cpu | cuda (default: cuda if available)")
    sub = ap.add_subparsers(dest="program", required=True)
    mods = {}
    for name, (mod, cfg_name, fn) in PROGRAMS.items():
        m = importlib.import_module(f"ddl25spring_amd.{mod}")
        mods[name] = (getattr(m, cfg_name), getattr(m, fn))
        _add_fields(sub.add_parser(name), mods[name][0])
    a = ap.parse_args(argv)
    cls, fn = mods[a.program]
    cfg = cls(**{f.name: getattr(a, f.name) for f in dataclasses.fields(cls)})
    from .runtime import dist as rdist
    ctx = rdist.init(device=a.device)
    try:
        out = fn(cfg, ctx)
        if a.program == "llm" and ctx.rank == 0:
            print(json.dumps({k: v for k, v in out.items() if k != "losses"}))
    finally:
        rdist.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
