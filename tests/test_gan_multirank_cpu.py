"""Federated DCGAN across ranks (BASELINE config 5, 'federated DCGAN on 2x MI355X'): the CLI program
under the launcher with 2 gloo ranks reproduces the single-process FedAvg of (G, D).

Reference aggregation template: lab/tutorial_1a/hfl_complete.py:336-390 (FedAvgServer)."""
import os
import subprocess
import sys

import torch

from ddl25spring_amd.runtime.launch import launch

ARGS = ["gan", "--clients", "2", "--rounds", "2", "--local-steps", "2", "--batch-size", "8",
        "--train-size", "64", "--ngf", "32", "--ndf", "32", "--seed", "3"]


def _env():
    env = dict(os.environ)
    env["PYTHONPATH"] = os.path.dirname(os.path.dirname(os.path.abspath(__file__))) + os.pathsep + \
        env.get("PYTHONPATH", "")
    env["OMP_NUM_THREADS"] = "2"
    return env


def test_gan_two_gloo_ranks_match_single_process(tmp_path):
    w1, w2 = tmp_path / "w1.pt", tmp_path / "w2.pt"
    cmd = [sys.executable, "-m", "ddl25spring_amd", "--device", "cpu", *ARGS]
    subprocess.run(cmd + ["--save", str(w1)], check=True, env=_env(), timeout=600)
    os.environ.update({k: v for k, v in _env().items() if k in ("PYTHONPATH", "OMP_NUM_THREADS")})
    res = launch(cmd + ["--save", str(w2)], world=2, log_dir=str(tmp_path / "logs"), timeout=600)
    assert res["returncode"] == 0, res
    a = torch.load(w1, weights_only=True)
    b = torch.load(w2, weights_only=True)
    assert a.shape == b.shape and a.numel() > 100_000
    torch.testing.assert_close(b, a, rtol=1e-5, atol=1e-6)
    # and FedAvg actually moved the weights away from the seeded init
    torch.manual_seed(3)
    from ddl25spring_amd.models.dcgan import Discriminator, Generator
    init = torch.cat([t.detach().reshape(-1) for t in list(Generator(100, 32).parameters()) +
                      list(Discriminator(32).parameters())])
    assert not torch.allclose(a[:init.numel()], init)
