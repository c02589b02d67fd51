"""Sharded checkpoint / resume (runtime/checkpoint.py): a DP x PP LLaMA job stopped after k steps
and restarted from its checkpoint ends bit-identical to an uninterrupted run (gloo ranks, CPU)."""
import json
import os
import tempfile

import pytest
import torch
import torch.multiprocessing as mp

TINY = dict(vocab_size=96, dmodel=32, num_heads=2, n_layers=4, ctx_size=16, batch_size=4,
            micro_batches=2, log_every=1)


def _llm_worker(rank, world, port, cfg_kw, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    from ddl25spring_amd.apps.llm import LLMConfig, train_llm
    from ddl25spring_amd.runtime import dist as rdist
    ctx = rdist.init(backend="gloo", device="cpu")
    res = train_llm(LLMConfig(**cfg_kw), ctx, log=None)
    torch.save({"losses": res["losses"], "resumed_from": res["resumed_from"]},
               os.path.join(out, f"res{rank}.pt"))
    rdist.shutdown()


def _run(world, port, cfg_kw, out):
    os.makedirs(out, exist_ok=True)
    mp.spawn(_llm_worker, args=(world, port, cfg_kw, out), nprocs=world, join=True)
    return [torch.load(os.path.join(out, f"res{r}.pt"), weights_only=True) for r in range(world)]


def _shards(d, step, world):
    return [torch.load(os.path.join(d, f"step{step:08d}", f"rank{r:05d}.pt"), weights_only=True)["state"]
            for r in range(world)]


def _assert_identical(a, b, path=""):
    if isinstance(a, torch.Tensor):
        assert torch.equal(a, b), path
    elif isinstance(a, dict):
        assert a.keys() == b.keys(), path
        for k in a:
            _assert_identical(a[k], b[k], f"{path}.{k}")
    elif isinstance(a, (list, tuple)):
        assert len(a) == len(b), path
        for i, (x, y) in enumerate(zip(a, b)):
            _assert_identical(x, y, f"{path}[{i}]")
    else:
        assert a == b, path


@pytest.mark.parametrize("dp_mode", ["ga", "wa"])
def test_llm_dp_pp_resume_is_bit_identical(dp_mode):
    cfg = dict(TINY, dp=2, pp=2, dp_mode=dp_mode, schedule="1f1b")
    port = 29971 if dp_mode == "ga" else 29975
    with tempfile.TemporaryDirectory() as d:
        full, part = os.path.join(d, "full"), os.path.join(d, "part")
        r_full = _run(4, port, dict(cfg, iters=5, ckpt_dir=full), os.path.join(d, "o1"))
        # "crash" after 2 steps (checkpoint committed at step 2), then restart for the full 5
        _run(4, port + 1, dict(cfg, iters=2, ckpt_dir=part), os.path.join(d, "o2"))
        assert json.load(open(os.path.join(part, "latest.json")))["step"] == 2
        r_res = _run(4, port + 2, dict(cfg, iters=5, ckpt_dir=part), os.path.join(d, "o3"))
        assert all(r["resumed_from"] == 2 for r in r_res)
        a, b = _shards(full, 5, 4), _shards(part, 5, 4)
        for r in range(4):
            _assert_identical(a[r], b[r], f"rank{r}")
        # the resumed run logged only steps 2..4, with exactly the uninterrupted run's losses
        for r in (1, 3):  # last stage of each pipeline
            tail = [x for x in r_full[r]["losses"] if x[0] >= 2]
            assert r_res[r]["losses"] == tail
        # older step directories were pruned; the step-2 shards are gone
        assert not os.path.exists(os.path.join(part, "step00000002"))


def test_checkpoint_rejects_mismatched_world(tmp_path):
    from ddl25spring_amd.runtime.checkpoint import ShardedCheckpoint

    class Ctx:
        rank, world = 0, 1

        def barrier(self):
            pass

    ck = ShardedCheckpoint(str(tmp_path), Ctx(), tag="a")
    ck.save(3, {"w": torch.arange(4.0), "n": 7})
    step, st = ck.load()
    assert step == 3 and st["n"] == 7 and torch.equal(st["w"], torch.arange(4.0))
    Ctx.world = 2
    with pytest.raises(ValueError, match="ranks"):
        ShardedCheckpoint(str(tmp_path), Ctx(), tag="a").latest()
    Ctx.world = 1
    with pytest.raises(ValueError, match="tag"):
        ShardedCheckpoint(str(tmp_path), Ctx(), tag="b").latest()


def _vfl_worker(rank, world, port, cfg_kw, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    torch.set_num_threads(1)
    from ddl25spring_amd.apps.vfl import VFLConfig, run_vfl
    from ddl25spring_amd.runtime import dist as rdist
    ctx = rdist.init(backend="gloo", device="cpu")
    res = run_vfl(VFLConfig(**cfg_kw), ctx, log=None)
    res.pop("real_data", None)
    torch.save(res, os.path.join(out, f"res{rank}.pt"))
    rdist.shutdown()


def test_splitnn_resume_is_bit_identical():
    cfg = dict(task="splitnn", parties=2, partition="balanced", batch_size=64)
    with tempfile.TemporaryDirectory() as d:
        full, part = os.path.join(d, "full"), os.path.join(d, "part")

        def run(port, kw, o):
            os.makedirs(o, exist_ok=True)
            mp.spawn(_vfl_worker, args=(3, port, dict(cfg, **kw), o), nprocs=3, join=True)
            return torch.load(os.path.join(o, "res0.pt"), weights_only=True)

        r_full = run(29981, dict(epochs=6, ckpt_dir=full), os.path.join(d, "o1"))
        run(29982, dict(epochs=3, ckpt_dir=part), os.path.join(d, "o2"))
        r_res = run(29983, dict(epochs=6, ckpt_dir=part), os.path.join(d, "o3"))
        assert r_res["resumed_from"] == 3
        a, b = _shards(full, 6, 3), _shards(part, 6, 3)
        for r in range(3):
            _assert_identical(a[r], b[r], f"rank{r}")
        assert r_res["test_accuracy"] == r_full["test_accuracy"]
        assert r_res["train_loss"] == r_full["train_loss"]


def test_federated_gan_resume_is_bit_identical(tmp_path):
    """Federated DCGAN over 2 gloo ranks (one client each): 3 rounds straight vs 1 round, stop,
    resume to 3 — the final global (G | D | BN) weights are bit-identical."""
    import subprocess
    import sys

    from ddl25spring_amd.runtime.launch import launch
    args = ["gan", "--clients", "2", "--local-steps", "2", "--batch-size", "8", "--train-size", "64",
            "--ngf", "16", "--ndf", "16", "--seed", "5"]
    cmd = [sys.executable, "-m", "ddl25spring_amd", "--device", "cpu", *args]
    env_keep = dict(os.environ)
    os.environ["OMP_NUM_THREADS"] = "2"
    try:
        full, part = tmp_path / "full", tmp_path / "part"
        r = launch(cmd + ["--rounds", "3", "--ckpt-dir", str(full), "--save", str(tmp_path / "a.pt")],
                   world=2, log_dir=str(tmp_path / "l1"), timeout=600)
        assert r["returncode"] == 0, r
        r = launch(cmd + ["--rounds", "1", "--ckpt-dir", str(part)], world=2,
                   log_dir=str(tmp_path / "l2"), timeout=600)
        assert r["returncode"] == 0, r
        r = launch(cmd + ["--rounds", "3", "--ckpt-dir", str(part), "--save", str(tmp_path / "b.pt")],
                   world=2, log_dir=str(tmp_path / "l3"), timeout=600)
        assert r["returncode"] == 0, r
    finally:
        os.environ.clear()
        os.environ.update(env_keep)
    a = torch.load(tmp_path / "a.pt", weights_only=True)
    b = torch.load(tmp_path / "b.pt", weights_only=True)
    assert torch.equal(a, b)
    _assert_identical(_shards(str(full), 3, 2), _shards(str(part), 3, 2))
