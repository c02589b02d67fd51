"""Homework 1 (reference lab/homework-1.ipynb) — every experiment of parts A and B.

Defaults of the notebook (L50-59): N=100 clients, lr=0.01, C=0.1, E=1, B=100, 10 rounds, IID,
seed=10. MNIST is the synthetic stand-in unless DDL_DATA_ROOT holds a torchvision copy.

  A1  FedSGD exchanging gradients vs weights (L132-230, L375-879). The notebook's
      FedSgdWeightServer exchanged gradients; here it is the real weight-exchanging
      FedSGD = FedAvg(E=1, B=inf), and the table shows both agree round by round.
  A2  number of clients N in {10, 50, 100} (L2144-2168) and client fraction C in {0.01, 0.1, 0.2}
      (L3391-3405): final accuracy and message counts for FedSGD and FedAvg.
  A3  local epochs E in {1, 2, 4} (L3494-3517), IID vs non-IID over 15 rounds (L3567-3591) and
      the lr = 0.001 / C = 0.5 non-IID stability run (L3641-3664): accuracy curves.
  B1  micro-batched GPipe pipeline, 3 stages x 3 micro-batches (L3723-3863) — 3 ranks.
  B2  DP x PP grid, 2 pipelines x 3 stages (L3919-4151; deadlocked in the reference)
      — 6 ranks, verified 1F1B schedule, collective sub-groups.

    python examples/homework_1.py --out lab_out/hw1 [--parts A1,A2,A3,B1,B2] [--quick]
"""
from __future__ import annotations

import subprocess
import sys

import pandas as pd

from _common import child_env, lineplot, outdir, parser, repo_root, save_table


def part_a1(H, cfg, out):
    rows = []
    for tag, n, iid, c, lr in (("N=100 IID C=0.5", cfg["n"], True, 0.5, 0.01),
                               ("N=50 non-IID C=0.2 lr=0.1", cfg["n50"], False, 0.2, 0.1)):
        sub = H.split(n, iid, 10)
        g = H.FedSgdGradientServer(lr, sub, c, 10).run(cfg["r5"]).as_df()
        w = H.FedSgdWeightServer(lr, sub, c, 10).run(cfg["r5"]).as_df()
        for (_, rg), (_, rw) in zip(g.iterrows(), w.iterrows()):
            rows.append({"Setting": tag, "Round": rg["Round"], "FedSGD (gradients)": rg["Test accuracy"],
                         "FedSGD (weights)": rw["Test accuracy"],
                         "Difference": rw["Test accuracy"] - rg["Test accuracy"]})
    df = pd.DataFrame(rows)
    save_table(df, out, "A1_fedsgd_gradients_vs_weights")
    return df


def part_a2(H, cfg, out):
    rows = []
    for n in cfg["ns"]:
        sub = H.split(n, True, 10)
        for name, srv in (("FedSGD", H.FedSgdGradientServer(0.01, sub, 0.1, 10)),
                          ("FedAvg", H.FedAvgServer(0.01, 100, sub, 0.1, 1, 10))):
            r = srv.run(cfg["r10"]).as_df().iloc[-1]
            rows.append({"Sweep": "N", "N": n, "C": 0.1, "Algorithm": name,
                         "Test accuracy": r["Test accuracy"], "Message count": r["Message count"]})
    sub = H.split(cfg["n"], True, 10)
    for c in (0.01, 0.1, 0.2):
        for name, srv in (("FedSGD", H.FedSgdGradientServer(0.01, sub, c, 10)),
                          ("FedAvg", H.FedAvgServer(0.01, 100, sub, c, 1, 10))):
            r = srv.run(cfg["r10"]).as_df().iloc[-1]
            rows.append({"Sweep": "C", "N": cfg["n"], "C": c, "Algorithm": name,
                         "Test accuracy": r["Test accuracy"], "Message count": r["Message count"]})
    df = pd.DataFrame(rows)
    save_table(df, out, "A2_clients_and_fraction")
    return df


def part_a3(H, cfg, out):
    sub = H.split(cfg["n"], True, 10)
    frames = []
    for e in (1, 2, 4):
        d = H.FedAvgServer(0.01, 100, sub, 0.1, e, 10).run(cfg["r10"]).as_df()
        d["Algorithm"] = f"FedAvg E={e}"
        frames.append(d)
    de = pd.concat(frames, ignore_index=True)
    save_table(de, out, "A3_local_epochs")
    lineplot(de, "Round", "Test accuracy", "Algorithm", out, "A3_local_epochs", "Local epochs E")
    frames = []
    for iid in (True, False):
        s = H.split(cfg["n"], iid, 10)
        for name, srv in (("FedSGD", H.FedSgdGradientServer(0.01, s, 0.1, 10)),
                          ("FedAvg", H.FedAvgServer(0.01, 100, s, 0.1, 1, 10))):
            d = srv.run(cfg["r15"]).as_df()
            d["Algorithm"] = f"{name} {'IID' if iid else 'non-IID'}"
            frames.append(d)
    di = pd.concat(frames, ignore_index=True)
    save_table(di, out, "A3_iid_vs_noniid")
    lineplot(di, "Round", "Test accuracy", "Algorithm", out, "A3_iid_vs_noniid", "IID vs non-IID")
    s = H.split(cfg["n"], False, 10)
    frames = []
    for name, srv in (("FedSGD", H.FedSgdGradientServer(0.001, s, 0.5, 10)),
                      ("FedAvg", H.FedAvgServer(0.001, 100, s, 0.5, 1, 10))):
        d = srv.run(cfg["r15"]).as_df()
        d["Algorithm"] = name
        frames.append(d)
    dl = pd.concat(frames, ignore_index=True)
    save_table(dl, out, "A3_lr0.001_C0.5_noniid")
    lineplot(dl, "Round", "Test accuracy", "Algorithm", out, "A3_lr0.001_C0.5_noniid",
             "non-IID, lr 0.001, C 0.5")
    return de, di, dl


def _llm(world, args, out, name, quick):
    cmd = [sys.executable, "-m", "ddl25spring_amd.runtime.launch", "-n", str(world), "--log-dir",
           str(out / name), "--timeout", "1800", "-m", "ddl25spring_amd", "llm", *args]
    if quick:
        cmd += ["--dmodel", "48", "--num-heads", "2", "--n-layers", "3", "--ctx-size", "32",
                "--vocab-size", "512", "--iters", "3", "--log-every", "1"]
    print("+", " ".join(cmd[1:]), flush=True)
    subprocess.run(cmd, check=True, cwd=repo_root(), env=child_env())


def main(argv=None):
    ap = parser(__doc__)
    ap.add_argument("--parts", default="A1,A2,A3,B1,B2")
    a = ap.parse_args(argv)
    out = outdir(a.out)
    parts = set(a.parts.split(","))
    from ddl25spring_amd.compat import hfl_complete as H
    cfg = dict(n=100, n50=50, ns=(10, 50, 100), r5=5, r10=10, r15=15)
    if a.quick:
        H.configure(n_train=2000, n_test=400)
        cfg = dict(n=10, n50=5, ns=(4, 10), r5=2, r10=2, r15=2)
    res = {}
    if "A1" in parts:
        res["A1"] = part_a1(H, cfg, out)
        print(res["A1"].to_string(index=False))
    if "A2" in parts:
        res["A2"] = part_a2(H, cfg, out)
        print(res["A2"].to_string(index=False))
    if "A3" in parts:
        res["A3"] = part_a3(H, cfg, out)
    if "B1" in parts:  # 3 stages x 2 layers, batch 3, 3 micro-batches, GPipe (all-F then all-B)
        _llm(3, ["--pp", "3", "--batch-size", "3", "--micro-batches", "3", "--schedule", "gpipe",
                 "--iters", "100"], out, "B1_gpipe", a.quick)
    if "B2" in parts:  # 2 pipelines x 3 stages, 1F1B
        _llm(6, ["--dp", "2", "--pp", "3", "--batch-size", "3", "--micro-batches", "3",
                 "--schedule", "1f1b", "--iters", "100"], out, "B2_dp2xpp3", a.quick)
    return res


if __name__ == "__main__":
    main(sys.argv[1:])
