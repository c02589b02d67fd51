"""End-to-end programs through the CLI and the launcher (gloo ranks on the CPU)."""
import json
import os
import sys
import tempfile

from ddl25spring_amd.cli import main
from ddl25spring_amd.runtime.launch import launch

TINY_LLM = ["--dmodel", "32", "--num-heads", "2", "--n-layers", "4", "--ctx-size", "16",
            "--vocab-size", "96", "--batch-size", "4", "--log-every", "1"]


def test_cli_fl_and_vfl_single_process(capsys):
    assert main(["--device", "cpu", "fl", "--model", "mnist_mlp", "--clients", "4",
                 "--client-fraction", "0.5", "--rounds", "2", "--train-size", "400",
                 "--test-size", "200", "--batch-size", "50", "--lr", "0.1"]) == 0
    out = capsys.readouterr().out
    assert "Test accuracy" in out and "Samples/s" in out
    assert main(["--device", "cpu", "vfl", "--task", "vflvae", "--epochs", "3"]) == 0


def _run(nproc, args, d):
    cmd = [sys.executable, "-m", "ddl25spring_amd", "--device", "cpu"] + args
    res = launch(cmd, nproc, log_dir=d, timeout=240)
    logs = [open(os.path.join(d, f"out{r}.txt")).read() for r in range(nproc)]
    if res["returncode"] != 0:
        # the full log of every rank (the abort reason of a dead rank is usually at its end)
        for r, lg in enumerate(logs):
            sys.stderr.write(f"===== rank {r} =====\n{lg}\n")
        raise AssertionError(f"launcher result {res}; rank logs on stderr")
    return logs


def test_llm_dp_pp_grid_via_launcher():
    with tempfile.TemporaryDirectory() as d:
        logs = _run(4, ["llm", "--dp", "2", "--pp", "2", "--micro-batches", "2", "--iters", "3"]
                    + TINY_LLM, d)
    summary = json.loads(logs[0].strip().splitlines()[-1])
    assert summary["tokens_per_s"] > 0
    # the loss is reported by the last stage of each pipeline (ranks 1 and 3)
    assert "stage 1] iter 2 loss" in logs[1] and "stage 1] iter 2 loss" in logs[3]


def test_llm_dp_weight_aggregation_via_launcher():
    with tempfile.TemporaryDirectory() as d:
        _run(2, ["llm", "--dp", "2", "--dp-mode", "wa", "--iters", "2"] + TINY_LLM, d)


def test_distributed_splitnn_via_launcher():
    with tempfile.TemporaryDirectory() as d:
        logs = _run(3, ["vfl", "--task", "splitnn", "--parties", "2", "--partition", "balanced",
                        "--epochs", "3"], d)
    assert "test_accuracy" in logs[0]
