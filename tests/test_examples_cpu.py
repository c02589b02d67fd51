"""Every lab script (examples/, the reference notebooks' equivalents) runs end to end in --quick
mode on the CPU and writes its tables and figures."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EX = os.path.join(ROOT, "examples")


@pytest.fixture(autouse=True)
def _examples_path(monkeypatch):
    monkeypatch.syspath_prepend(EX)


def _run(mod, tmp_path, *args):
    import importlib
    m = importlib.import_module(mod)
    return m.main(["--quick", "--out", str(tmp_path), *args])


def test_lab_1a(tmp_path):
    df = _run("lab_1a_hfl", tmp_path)
    assert set(df["Algorithm"]) >= {"FedAvg"} and len(df) == 6
    assert (tmp_path / "tutorial_1a.png").exists() and (tmp_path / "tutorial_1a.csv").exists()


def test_homework_1_part_a(tmp_path):
    res = _run("homework_1", tmp_path, "--parts", "A1,A2,A3")
    a1 = res["A1"]
    assert (a1["Difference"].abs() < 5.0).all()  # FedSGD exchanging gradients == weights
    assert len(res["A2"]) == 10
    for name in ("A3_local_epochs", "A3_iid_vs_noniid", "A3_lr0.001_C0.5_noniid"):
        assert (tmp_path / f"{name}.png").exists()


@pytest.mark.slow
def test_homework_1_part_b(tmp_path):
    _run("homework_1", tmp_path, "--parts", "B1")
    assert (tmp_path / "B1_gpipe" / "out2.txt").exists()


def test_lab_1b_dp_pp(tmp_path):
    df = _run("lab_1b_dp_pp", tmp_path, "--runs", "intro,pp_gpipe")
    assert set(df["Run"]) == {"intro", "pp_gpipe"}
    assert (tmp_path / "tutorial_1b_losses.png").exists()


def test_lab_2a(tmp_path):
    df = _run("lab_2a_generative", tmp_path)
    assert len(df) == 3 and df["Best test accuracy"].between(0, 100).all()


def test_lab_2b_and_homework_2(tmp_path):
    curve, acc = _run("lab_2b_vfl", tmp_path)
    assert 0.0 <= acc <= 1.0 and len(curve) == 5
    res = _run("homework_2", tmp_path)
    assert list(res["ex1"]["Seed"]) == [42, 43, 44]
    assert list(res["ex2"]["Parties"]) == [2, 4, 6, 8]
    assert len(res["ex3"]) == 10
    for name in ("ex1_permutations", "ex2_parties", "ex3_vflvae_loss"):
        assert (tmp_path / f"{name}.png").exists()
