"""Shared helpers for the lab scripts: output directory, quick mode, tables and line plots.

The reference's notebooks plot with seaborn (``sns.lineplot(x="Round", y="Test accuracy",
hue="Algorithm")``, horizontal-federated-learning.ipynb:502-507); seaborn is not installed here,
so the same long-format DataFrames are drawn with matplotlib (Agg backend, PNG files) and saved
as CSV next to the figure.
"""
from __future__ import annotations

import argparse
import os
import sys
from pathlib import Path

_ROOT = str(Path(__file__).resolve().parent.parent)
if _ROOT not in sys.path:  # run from a checkout: `python examples/<script>.py`
    sys.path.insert(0, _ROOT)


def parser(doc: str) -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(description=doc, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--out", default="lab_out", help="directory for tables (CSV) and figures (PNG)")
    ap.add_argument("--quick", action="store_true",
                    help="tiny data / few rounds: checks the pipeline end to end in seconds")
    return ap


def outdir(path: str) -> Path:
    p = Path(path)
    p.mkdir(parents=True, exist_ok=True)
    return p


def save_table(df, out: Path, name: str) -> Path:
    f = out / f"{name}.csv"
    df.to_csv(f, index=False)
    return f


def lineplot(df, x: str, y: str, hue: str, out: Path, name: str, title: str = "") -> Path:
    """seaborn-style ``lineplot(data=df, x=x, y=y, hue=hue)`` with matplotlib."""
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    fig, ax = plt.subplots(figsize=(6, 4))
    for key, g in df.groupby(hue, sort=False):
        ax.plot(g[x], g[y], marker="o", ms=3, label=str(key))
    ax.set_xlabel(x)
    ax.set_ylabel(y)
    if title:
        ax.set_title(title)
    ax.legend(title=hue, fontsize=8)
    ax.grid(alpha=0.3)
    fig.tight_layout()
    f = out / f"{name}.png"
    fig.savefig(f, dpi=110)
    plt.close(fig)
    return f


def repo_root() -> str:
    return str(Path(__file__).resolve().parent.parent)


def child_env() -> dict:
    env = dict(os.environ)
    env["PYTHONPATH"] = repo_root() + os.pathsep + env.get("PYTHONPATH", "")
    return env
