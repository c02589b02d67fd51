"""Tutorial 2a — centralized heart-disease model and the tabular VAE (reference
lab/tutorial_2a/centralized.py and generative-modeling.py).

  centralized  HeartDiseaseNN, full-batch AdamW, 49 epochs, best test accuracy kept (the
               reference's ``best_params = net.state_dict()`` aliased the live weights, SURVEY Q9;
               here it is a deep copy)
  vae          Autoencoder(31, 48, 32, 16) + customLoss (MSE(sum) + KL), Adam 1e-3, 200 epochs,
               then "train on synthetic, test on real": HeartDiseaseNN trained on real vs on
               sampled rows, both tested on the real test split

heart.csv is read from the reference checkout when it is mounted, else a synthetic table of the
same schema is used (data/heart.py).

    python examples/lab_2a_generative.py --out lab_out/2a [--quick]
"""
from __future__ import annotations

import sys

import pandas as pd

from _common import outdir, parser, save_table


def main(argv=None):
    a = parser(__doc__).parse_args(argv)
    out = outdir(a.out)
    from ddl25spring_amd.apps.vfl import VFLConfig, run_vfl
    from ddl25spring_amd.runtime import dist as rdist
    ctx = rdist.init()
    c = run_vfl(VFLConfig(task="centralized", epochs=5 if a.quick else 49), ctx, log=None)
    v = run_vfl(VFLConfig(task="vae", epochs=3 if a.quick else 200), ctx, log=None)
    df = pd.DataFrame([
        {"Experiment": "centralized HeartDiseaseNN", "Best test accuracy": c["best_test_accuracy"],
         "Real heart.csv": c["real_data"]},
        {"Experiment": "VAE: classifier trained on real rows", "Best test accuracy": v["real_trained_acc"],
         "Real heart.csv": v["real_data"]},
        {"Experiment": "VAE: classifier trained on synthetic rows",
         "Best test accuracy": v["synthetic_trained_acc"], "Real heart.csv": v["real_data"]},
    ])
    print(df.to_string(index=False))
    print(f"VAE final loss {v['final_loss']:.2f}")
    save_table(df, out, "tutorial_2a")
    return df


if __name__ == "__main__":
    main(sys.argv[1:])
