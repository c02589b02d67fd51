"""Tutorial 1b — data and pipeline parallelism on the small LLaMA (reference lab/tutorial_1b:
primer/intro.py, DP/gradient_aggr/intro_DP_GA.py, DP/weight_aggr/intro_DP_WA.py,
PP/1F1B/intro_PP_1F1B.py, intro_PP_1F1B_MB.py, intro_PP_1F1B_MP.py and their run*.sh launchers).

Each script of the tutorial is one configuration of ``python -m ddl25spring_amd llm`` under the
launcher (one rank per GPU over RCCL, or gloo ranks on the CPU; per-rank logs out{rank}.txt like
the reference's run.sh, and a crashed rank takes the whole job down):

  intro        dp 1 pp 1                              (primer/intro.py)
  dp_ga        dp 3, gradient all-reduce              (intro_DP_GA.py: 3 ranks)
  dp_wa        dp 3, weight averaging written back    (intro_DP_WA.py; the reference never wrote
                                                       the average back)
  pp_naive     pp 3, one batch                        (intro_PP_1F1B.py)
  pp_gpipe     pp 3, 3 micro-batches, all-F-all-B     (intro_PP_1F1B_MB.py)
  pp_1f1b      pp 3, 3 micro-batches, 1F1B            (the schedule intro_PP_1F1B_MP.py attempted)
  dp_x_pp      2 pipelines x 3 stages                 (intro_PP_1F1B_MP.py; deadlocked there)

    python examples/lab_1b_dp_pp.py --out lab_out/1b [--runs intro,dp_ga,...] [--iters 500] [--quick]
"""
from __future__ import annotations

import re
import subprocess
import sys

import pandas as pd

from _common import child_env, lineplot, outdir, parser, repo_root, save_table

RUNS = {
    "intro": (1, []),
    "dp_ga": (3, ["--dp", "3", "--dp-mode", "ga"]),
    "dp_wa": (3, ["--dp", "3", "--dp-mode", "wa"]),
    "pp_naive": (3, ["--pp", "3", "--micro-batches", "1", "--schedule", "naive"]),
    "pp_gpipe": (3, ["--pp", "3", "--micro-batches", "3", "--schedule", "gpipe"]),
    "pp_1f1b": (3, ["--pp", "3", "--micro-batches", "3", "--schedule", "1f1b"]),
    "dp_x_pp": (6, ["--dp", "2", "--pp", "3", "--micro-batches", "3", "--schedule", "1f1b"]),
}
_LOSS = re.compile(r"iter (\d+) loss ([0-9.eE+-]+)")


def main(argv=None):
    ap = parser(__doc__)
    ap.add_argument("--runs", default=",".join(RUNS))
    ap.add_argument("--iters", type=int, default=500)
    ap.add_argument("--batch-size", type=int, default=3)
    a = ap.parse_args(argv)
    out = outdir(a.out)
    rows = []
    for name in a.runs.split(","):
        world, args = RUNS[name]
        log_dir = out / name
        cmd = [sys.executable, "-m", "ddl25spring_amd.runtime.launch", "-n", str(world),
               "--log-dir", str(log_dir), "--timeout", "3600", "-m", "ddl25spring_amd", "llm", *args,
               "--batch-size", str(a.batch_size), "--iters", str(a.iters),
               "--log-every", str(max(1, a.iters // 50))]
        if a.quick:
            cmd += ["--dmodel", "48", "--num-heads", "2", "--n-layers", "3", "--ctx-size", "32",
                    "--vocab-size", "512", "--iters", "4", "--log-every", "1"]
        print("+", " ".join(cmd[1:]), flush=True)
        subprocess.run(cmd, check=True, cwd=repo_root(), env=child_env())
        # the loss is known on the last stage of each pipeline: rank pp-1 of pipeline 0
        pp = int(args[args.index("--pp") + 1]) if "--pp" in args else 1
        text = (log_dir / f"out{pp - 1}.txt").read_text()
        for it, loss in _LOSS.findall(text):
            rows.append({"Run": name, "Iteration": int(it), "Loss": float(loss)})
    df = pd.DataFrame(rows)
    save_table(df, out, "tutorial_1b_losses")
    if len(df):
        lineplot(df, "Iteration", "Loss", "Run", out, "tutorial_1b_losses", "LLaMA-288d training loss")
    return df


if __name__ == "__main__":
    main(sys.argv[1:])
