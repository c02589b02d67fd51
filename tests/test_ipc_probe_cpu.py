"""probe_ipc_threshold agreement (runtime/dist.py): a peer path that returns wrong sums, or raises,
on ONE rank must send every rank to the same fallback without mismatched collectives (gloo, 2 ranks,
a fake peer-read object standing in for runtime/ipc.IpcAllReduce)."""
import json
import os
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ddl25spring_amd.runtime import dist as rdist


class _FakeIpc:
    """Stands in for the peer-read all-reduce, which is NOT a process-group collective: it returns
    the probe's expected sum (sum of rank + 1) without talking to the group, or on one rank a wrong
    sum / a peer timeout."""

    def __init__(self, rank, world, bad_rank, how):
        self.rank, self.world, self.bad_rank, self.how = rank, world, bad_rank, how
        self.cap = 1 << 20
        self.closed = False

    def all_reduce(self, t):
        if self.rank == self.bad_rank and self.how == "raise":
            raise RuntimeError("peer timed out")
        if t[0].item() == float(self.rank + 1):  # the correctness probe's input
            t.fill_(float(self.world * (self.world + 1) // 2))
        if self.rank == self.bad_rank and self.how == "wrong":
            t.add_(1.0)

    def check(self):
        pass

    def close(self):
        self.closed = True


def _worker(rank, world, port, out_dir, bad_rank, how):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ctx = rdist.DistContext(rank, world, rank, torch.device("cpu"), "gloo")
        ctx.ipc = _FakeIpc(rank, world, bad_rank, how)
        thr = rdist.probe_ipc_threshold(ctx, sizes=(16 << 10, 64 << 10, 256 << 10), iters=1)
        # the group is still usable: one more collective completes with the right value
        x = torch.ones(4)
        dist.all_reduce(x)
        with open(os.path.join(out_dir, f"r{rank}.json"), "w") as f:
            json.dump({"thr": thr, "ipc_none": ctx.ipc is None, "err": ctx.ipc_policy.get("error", ""),
                       "after": x.tolist()}, f)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("how", ["wrong", "raise"])
def test_probe_one_bad_rank_all_fall_back(how):
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(2, 29971 + (how == "raise"), d, 1, how), nprocs=2, join=True)
        res = [json.load(open(os.path.join(d, f"r{r}.json"))) for r in range(2)]
    for r in res:
        assert r["thr"] == 0 and r["ipc_none"], r
        assert r["after"] == [2.0] * 4
    assert "wrong sums" in res[1]["err"] or "timed out" in res[1]["err"]


def test_probe_healthy_peer_path_keeps_a_threshold_policy():
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(2, 29975, d, -1, "none"), nprocs=2, join=True)
        res = [json.load(open(os.path.join(d, f"r{r}.json"))) for r in range(2)]
    assert res[0]["thr"] == res[1]["thr"]  # the decision is identical on every rank
    assert res[0]["err"] == "" and res[1]["err"] == ""
