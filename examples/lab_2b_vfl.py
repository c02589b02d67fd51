"""Tutorial 2b — vertical federated learning, split-NN on the heart-disease table (reference
lab/tutorial_2b/lab-vfl.ipynb and vfl.py).

4 parties own the raw-column feature partition (vfl.py:116-141: one-hot widths [7, 4, 6, 13]),
each a BottomModel(f, 2f); the label holder's TopModel joins the cut-layer activations. AdamW,
300 epochs, batch 64, the 821 / 204 row split (vfl.py:150-152). The notebook reports 86.76 % test
accuracy (lab-vfl.ipynb:572). ``--parity`` reproduces the reference's quirks (bottom models never
trained, zero_grad once per epoch, dropout active at test: SURVEY Q5/Q6/Q8).

    python examples/lab_2b_vfl.py --out lab_out/2b [--parity] [--quick]

One party per process (the label holder on rank 0, cut-layer tensors over RCCL / gloo P2P):
    python -m ddl25spring_amd.runtime.launch -n 5 -m ddl25spring_amd vfl --task splitnn --parties 4
"""
from __future__ import annotations

import sys

import pandas as pd
import torch

from _common import lineplot, outdir, parser, save_table


def train_splitnn(partition: str, parties: int, epochs: int, seed: int = 42, perm_seed: int = 42,
                  parity: bool = False):
    """-> (per-epoch DataFrame, test accuracy, test loss) of one split-NN run (the notebook's cell)."""
    import numpy as np
    from ddl25spring_amd.compat import vfl as V
    from ddl25spring_amd.models.tabular import BottomModel, VFLNetwork
    df, _ = V.load_heart()
    torch.manual_seed(seed)
    np.random.seed(seed)
    X, Y = V.vfl_frame(df)
    cols = list(X.columns)
    if partition == "raw":
        feats = V.partition_raw_columns(list(df.columns), cols, parties)
    elif partition == "random":
        feats = V.partition_random(cols, parties, perm_seed)
    else:
        feats = V.partition_balanced(cols, parties)
    Xtr, Xte = V.row_split(X)
    Ytr, Yte = V.row_split(Y)
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    net = VFLNetwork([BottomModel(len(f), 2 * len(f)) for f in feats], 2, parity=parity).to(dev)
    hist = net.train_with_settings(epochs, 64, parties, feats, Xtr, Ytr)
    acc, loss = net.test(Xte, Yte)
    curve = pd.DataFrame({"Epoch": range(1, len(hist) + 1), "Loss": [h[0] for h in hist],
                          "Train accuracy": [h[1] for h in hist]})
    return curve, float(acc), float(loss)


def main(argv=None):
    ap = parser(__doc__)
    ap.add_argument("--parity", action="store_true")
    a = ap.parse_args(argv)
    out = outdir(a.out)
    curve, acc, loss = train_splitnn("raw", 4, 5 if a.quick else 300, parity=a.parity)
    curve["Run"] = "split-NN, 4 parties"
    print(curve.tail(3).to_string(index=False))
    print(f"test accuracy {100 * acc:.2f} %  (published 86.76 %), test loss {loss:.3f}")
    save_table(curve, out, "tutorial_2b_curve")
    lineplot(curve, "Epoch", "Loss", "Run", out, "tutorial_2b_loss", "VFL split-NN training loss")
    return curve, acc


if __name__ == "__main__":
    main(sys.argv[1:])
