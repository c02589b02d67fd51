"""Launcher: env contract, per-rank logs, kill-all on the first failure, global timeout."""
import os
import sys
import tempfile
import textwrap

from ddl25spring_amd.runtime.launch import launch

OK = textwrap.dedent("""
    import os, torch, torch.distributed as dist
    dist.init_process_group("gloo")
    t = torch.ones(1) * (dist.get_rank() + 1)
    dist.all_reduce(t)
    print("rank", os.environ["RANK"], "of", os.environ["WORLD_SIZE"], "sum", int(t.item()), flush=True)
    dist.destroy_process_group()
""")

FAIL = textwrap.dedent("""
    import os, sys, torch.distributed as dist
    if os.environ["RANK"] == "1":
        sys.exit(3)
    dist.init_process_group("gloo")   # rank 0 would wait for rank 1 forever
    dist.barrier()
""")


def _script(d, body):
    p = os.path.join(d, "job.py")
    with open(p, "w") as f:
        f.write(body)
    return p


def test_launch_success_and_logs():
    with tempfile.TemporaryDirectory() as d:
        res = launch([sys.executable, _script(d, OK)], 3, log_dir=d, timeout=120)
        assert res["returncode"] == 0 and res["codes"] == [0, 0, 0]
        for r in range(3):
            txt = open(os.path.join(d, f"out{r}.txt")).read()
            assert f"rank {r} of 3 sum 6" in txt


def test_launch_kills_peers_on_failure():
    with tempfile.TemporaryDirectory() as d:
        res = launch([sys.executable, _script(d, FAIL)], 2, log_dir=d, timeout=120)
    assert res["returncode"] == 3 and res["failed_rank"] == 1
    assert res["elapsed"] < 60  # rank 0 was taken down, not left hanging
    assert res["codes"][0] is not None


def test_launch_timeout():
    with tempfile.TemporaryDirectory() as d:
        res = launch([sys.executable, "-c", "import time; time.sleep(60)"], 2, timeout=2)
    assert res["returncode"] == 124 and res["failed_rank"] == -1
