"""Tutorial 1a — horizontal federated learning (reference lab/tutorial_1a/
horizontal-federated-learning.ipynb, solution hfl_complete.py).

The notebook's three demo runs, unchanged API (``from ddl25spring_amd.compat.hfl_complete import *``):
  CentralizedServer(0.5, 1024, 42).run(5)                                 (ipynb L323-326)
  FedSgdGradientServer(0.02, split(100, True, 42), 0.2, 42).run(5)        (ipynb L418-421)
  FedAvgServer(0.02, 200, split(100, True, 42), 0.2, 2, 42).run(5)        (ipynb L483-486)
then the accuracy-per-round line plot by algorithm (ipynb L502-507).

    python examples/lab_1a_hfl.py --out lab_out/1a [--quick]
"""
from __future__ import annotations

import sys

import pandas as pd

from _common import lineplot, outdir, parser, save_table


def main(argv=None):
    a = parser(__doc__).parse_args(argv)
    out = outdir(a.out)
    from ddl25spring_amd.compat import hfl_complete as H
    rounds, n = 5, 100
    if a.quick:
        H.configure(n_train=3000, n_test=500)
        rounds, n = 2, 10
    results = [
        H.CentralizedServer(0.5, 1024, 42).run(rounds),
        H.FedSgdGradientServer(0.02, H.split(n, True, 42), 0.2, 42).run(rounds),
        H.FedAvgServer(0.02, 200, H.split(n, True, 42), 0.2, 2, 42).run(rounds),
    ]
    df = pd.concat([r.as_df() for r in results], ignore_index=True)
    print(df.to_string(index=False))
    save_table(df, out, "tutorial_1a")
    lineplot(df, "Round", "Test accuracy", "Algorithm", out, "tutorial_1a", "Tutorial 1a")
    return df


if __name__ == "__main__":
    main(sys.argv[1:])
