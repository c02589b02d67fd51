"""Peer-read all-reduce over hipIPC-mapped uncached buffers (csrc/kernels/ipc_allreduce.hip).

The test box has one GPU, so the ranks share it: every rank still maps every other rank's buffer
through hipIpcOpenMemHandle from a different process and the kernels synchronise through the
peers' signal words, exactly as on an 8-GPU node (where the loads cross xGMI instead)."""
import os
import tempfile

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _worker(rank, world, port, out, sizes, two_shot_bytes):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import torch.distributed as dist
    from ddl25spring_amd.runtime.ipc import IpcAllReduce
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    ar = IpcAllReduce(rank, world, dev, capacity=max(sizes) * 4, two_shot_bytes=two_shot_bytes,
                      nblocks=8, timeout_s=10.0)
    res = {}
    for rep in range(3):  # parity slots and the device epoch advance across calls
        for n in sizes:
            g = torch.Generator().manual_seed(1000 * rep + 7 * n + rank)
            x = torch.randn(n, generator=g).to(dev)
            ar.all_reduce(x)
            res[(rep, n)] = x.cpu()
    # back-to-back calls without a host sync in between: a fast rank runs whole calls ahead of a
    # slow one, so the barrier's epoch compare must be wrap-safe monotonic, not equality
    xs = [torch.full((777 + 64 * i,), float((rank + 1) * (i + 1)), device=dev) for i in range(8)]
    torch.cuda.synchronize()
    for t in xs:
        ar.all_reduce(t)
    res["b2b"] = [t.cpu() for t in xs]
    # graph-captured calls replay with the device-resident epoch
    x = torch.full((4099,), float(rank + 1), device=dev)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ar.all_reduce(x)
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        ar.all_reduce(x)
    x.fill_(float(rank + 1))
    dist.barrier()
    graph.replay()
    res["graph"] = x.cpu()
    ar.check()
    torch.save(res, os.path.join(out, f"r{rank}.pt"))
    dist.barrier()
    ar.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,two_shot_bytes", [(2, 1 << 30), (3, 1 << 30), (4, 256)],
                         ids=["2ranks-oneshot", "3ranks-oneshot", "4ranks-twoshot"])
def test_ipc_allreduce_matches_sum(cuda, world, two_shot_bytes):
    sizes = [1, 5, 1000, 4099, 65536 + 3]
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, 29751 + world, d, sizes, two_shot_bytes), nprocs=world,
                 join=True)
        outs = [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True) for r in range(world)]
    for rep in range(3):
        for n in sizes:
            want = sum(torch.randn(n, generator=torch.Generator().manual_seed(1000 * rep + 7 * n + r))
                       for r in range(world))
            for r in range(world):
                got = outs[r][(rep, n)]
                assert torch.equal(got, outs[0][(rep, n)]), "ranks disagree"  # bit-identical
                assert torch.allclose(got, want, rtol=1e-5, atol=1e-5)
    tot = float(sum(range(1, world + 1)))
    for r in range(world):
        assert torch.equal(outs[r]["graph"], torch.full((4099,), tot))
        for i, t in enumerate(outs[r]["b2b"]):
            assert torch.equal(t, torch.full((777 + 64 * i,), tot * (i + 1))), (r, i)


def _policy_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import torch.distributed as dist
    from ddl25spring_amd.runtime import dist as rdist
    from ddl25spring_amd.runtime.ipc import IpcAllReduce
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    ctx = rdist.DistContext(rank, world, rank, dev, "gloo")
    ctx.ipc = IpcAllReduce(rank, world, dev, capacity=1 << 20, nblocks=8, timeout_s=10.0)
    thr = rdist.probe_ipc_threshold(ctx, sizes=(16 << 10, 256 << 10, 1 << 20), iters=2)
    x = torch.full((50000,), float(rank + 1), device=dev)  # 200 KB: either path, per the policy
    ctx.all_reduce(x)
    torch.save({"thr": thr, "policy": ctx.ipc_policy, "x": x.cpu(),
                "path": rdist.allreduce_path(ctx, x.numel() * 4)}, os.path.join(out, f"p{rank}.pt"))
    dist.barrier()
    if ctx.ipc is not None:
        ctx.ipc.close()
    dist.destroy_process_group()


def test_ipc_threshold_probe_agrees_across_ranks(cuda):
    """The peer-read vs process-group all-reduce crossover probe (runtime/dist.py): every rank
    takes the same decision from the all-reduced timings, and the policy's all_reduce sums
    correctly on whichever path it chose (2 ranks sharing the GPU; gloo stands in for RCCL)."""
    from ddl25spring_amd.runtime.launch import free_port
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_policy_worker, args=(world, free_port(), d), nprocs=world, join=True,
                           start_method="spawn")
        res = [torch.load(os.path.join(d, f"p{r}.pt"), weights_only=True) for r in range(world)]
    assert res[0]["thr"] == res[1]["thr"] and res[0]["thr"] in (0, 16 << 10, 256 << 10, 1 << 20)
    assert res[0]["policy"]["probe_ms"] == res[1]["policy"]["probe_ms"]
    for r in res:
        assert torch.equal(r["x"], torch.full((50000,), 3.0))
        assert r["path"] == ("ipc" if r["thr"] >= 200000 else "gloo")


def _fedavg_worker(rank, world, port, out_path, P):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import torch.distributed as dist
    from ddl25spring_amd.fl.aggregate import MeanAggregator
    from ddl25spring_amd.runtime import dist as rdist
    from ddl25spring_amd.runtime.ipc import IpcAllReduce
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    ctx = rdist.DistContext(rank, world, rank, dev, "gloo")
    ctx.ipc = IpcAllReduce(rank, world, dev, capacity=16 << 20, nblocks=16, timeout_s=20.0)
    g = torch.Generator().manual_seed(11)
    rows = torch.randn(world, P, generator=g)
    coef = torch.rand(world, generator=g)
    coef /= coef.sum()
    agg = MeanAggregator(ordered=True)
    out = torch.empty(P, device=dev)
    agg(ctx, rows[rank:rank + 1].to(dev), coef[rank:rank + 1].to(dev), out)  # this rank's one client
    desc = agg.describe(ctx)
    ipc, ctx.ipc = ctx.ipc, None  # the all-gather fallback of the same reduction, for comparison
    out_g = torch.empty(P, device=dev)
    agg(ctx, rows[rank:rank + 1].to(dev), coef[rank:rank + 1].to(dev), out_g)
    ctx.ipc = ipc
    torch.save({"out": out.cpu(), "gather": out_g.cpu(), "desc": desc}, os.path.join(out_path, f"f{rank}.pt"))
    dist.barrier()
    ctx.ipc.check()
    ctx.ipc.close()
    dist.destroy_process_group()


def test_ipc_ordered_fedavg_mean_bitwise_single_process(cuda):
    """The 8-GPU headline's ordered FedAvg reduction (fl/aggregate.MeanAggregator) on the peer-read
    kernel: 4 ranks with one client each (sharing the GPU) give bitwise the single-process 4-slot
    weighted sum, on a vector of 5M floats (two-shot path, three slot-sized chunks)."""
    from ddl25spring_amd.ops import functional as Fn
    from ddl25spring_amd.runtime.launch import free_port
    world, P = 4, 5_000_003
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_fedavg_worker, args=(world, free_port(), d, P), nprocs=world, join=True,
                           start_method="spawn")
        res = [torch.load(os.path.join(d, f"f{r}.pt"), weights_only=True) for r in range(world)]
    g = torch.Generator().manual_seed(11)
    rows = torch.randn(world, P, generator=g)
    coef = torch.rand(world, generator=g)
    coef /= coef.sum()
    ref = torch.empty(P, device=cuda)
    Fn.weighted_sum(rows.to(cuda), coef.to(cuda), ref)
    ref = ref.cpu()
    for r in res:
        assert r["desc"] == "ipc peer-read rank-ordered sum"
        bad = (r["out"] != ref).nonzero().flatten()
        badg = (r["gather"] != ref).nonzero().flatten()
        assert bad.numel() == 0 and badg.numel() == 0, (bad.numel(), bad[:8].tolist(), badg.numel(),
                                                        (r["out"] - ref).abs().max().item())


def _bucket_worker(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import torch.distributed as dist
    from ddl25spring_amd.parallel.dp import GradBucketer, average_weights
    from ddl25spring_amd.runtime import dist as rdist
    from ddl25spring_amd.runtime.ipc import IpcAllReduce
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    ctx = rdist.DistContext(rank, world, rank, dev, "gloo")
    ctx.ipc = IpcAllReduce(rank, world, dev, capacity=1 << 20, nblocks=8, timeout_s=20.0)
    ctx.ipc_max_bytes = 1 << 20
    calls = []
    inner = ctx.ipc.all_reduce
    ctx.ipc.all_reduce = lambda t: (calls.append(t.numel()), inner(t))[1]
    torch.manual_seed(5)
    m = torch.nn.Sequential(torch.nn.Linear(64, 128), torch.nn.ReLU(), torch.nn.Linear(128, 10)).to(dev)
    g = torch.Generator().manual_seed(100 + rank)
    x, y = torch.randn(32, 64, generator=g).to(dev), torch.randint(0, 10, (32,), generator=g).to(dev)
    torch.nn.functional.cross_entropy(m(x), y).backward()
    local = [p.grad.detach().cpu().clone() for p in m.parameters()]
    for p in m.parameters():
        p.grad = None
    gb = GradBucketer(m, ctx, bucket_mb=0.02)  # several buckets, each below the 1 MiB crossover
    gb.zero_grad()
    torch.nn.functional.cross_entropy(m(x), y).backward()
    gb.finish()
    synced = [p.grad.detach().cpu().clone() for p in m.parameters()]
    nb = len(gb.buckets)
    with torch.no_grad():
        for p in m.parameters():
            p.add_(float(rank))
    average_weights(m, ctx)
    w = [p.detach().cpu().clone() for p in m.parameters()]
    torch.cuda.synchronize()
    ctx.ipc.check()
    torch.save({"local": local, "synced": synced, "calls": calls, "buckets": nb, "w": w},
               os.path.join(out_path, f"b{rank}.pt"))
    dist.barrier()
    ctx.ipc.close()
    dist.destroy_process_group()


def test_grad_bucketer_takes_peer_read_allreduce_below_crossover(cuda):
    """DP gradient buckets (parallel/dp.GradBucketer) and DP-WA below the measured crossover run
    the peer-read all-reduce (runtime/ipc.py) instead of RCCL: 2 ranks sharing the GPU, every
    bucket and the weight average on the peer path, gradients = the mean of the ranks' local
    gradients, bitwise equal on both ranks."""
    from ddl25spring_amd.runtime.launch import free_port
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_bucket_worker, args=(world, free_port(), d), nprocs=world, join=True,
                           start_method="spawn")
        res = [torch.load(os.path.join(d, f"b{r}.pt"), weights_only=True) for r in range(world)]
    nb = res[0]["buckets"]
    assert nb >= 2
    for r in res:
        assert len(r["calls"]) == nb + 1, r["calls"]  # every bucket + the DP-WA flat vector
    for i in range(len(res[0]["synced"])):
        want = (res[0]["local"][i] + res[1]["local"][i]) / 2
        assert torch.equal(res[0]["synced"][i], res[1]["synced"][i])
        assert torch.allclose(res[0]["synced"][i], want, rtol=1e-5, atol=1e-6)
        assert torch.equal(res[0]["w"][i], res[1]["w"][i])
