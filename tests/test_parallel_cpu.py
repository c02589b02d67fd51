"""Schedules, pipeline / data parallelism and the DP x PP grid on the CPU gloo backend."""
import os
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ddl25spring_amd.models.llama import LLama, causalLLMLoss, split_stages
from ddl25spring_amd.parallel import schedule as S

TINY = dict(vocab_size=96, dmodel=32, num_heads=2, n_layers=4, ctx_size=16)


@pytest.mark.parametrize("kind", ["gpipe", "1f1b", "naive"])
@pytest.mark.parametrize("stages", [1, 2, 3, 4])
@pytest.mark.parametrize("micro", [1, 2, 3, 5, 8])
def test_schedules_verify(kind, stages, micro):
    acts = S.make(kind, stages, micro)
    for s in range(stages):
        ops = [a for a in acts if a.stage == s]
        assert sorted(a.mb for a in ops if a.op == S.FWD) == list(range(micro))
        assert sorted(a.mb for a in ops if a.op == S.BWD) == list(range(micro))
    if kind == "1f1b":  # bounded activation memory: at most S - s in flight on stage s
        for s in range(stages):
            live = peak = 0
            for a in (a for a in acts if a.stage == s):
                live += (a.op == S.FWD) - (a.op == S.BWD)
                peak = max(peak, live)
            assert peak <= max(1, min(stages - s, micro))


def test_verifier_catches_reference_deadlock():
    """The reference's DPxPP schedule: stage 1 runs 1F1B, stage 2 receives ALL micro-batches
    before computing (intro_PP_1F1B_MP.py:86-157) -> deadlock at iteration 0 (out_MP*.txt)."""
    A = S.Action
    M = 3
    acts = []
    for m in range(M):
        acts += [A(0, S.FWD, m, -1, -1), A(0, S.SEND_ACT, m, 1, -1)]
    for m in reversed(range(M)):
        acts += [A(0, S.RECV_GRAD, m, 1, -1), A(0, S.BWD, m, -1, -1)]
    # stage 1: 1F1B-ish, wants grad of mb0 after sending act of mb1
    acts += [A(1, S.RECV_ACT, 0, 0, -1), A(1, S.FWD, 0, -1, -1), A(1, S.SEND_ACT, 0, 2, -1),
             A(1, S.RECV_ACT, 1, 0, -1), A(1, S.FWD, 1, -1, -1), A(1, S.SEND_ACT, 1, 2, -1),
             A(1, S.RECV_GRAD, 0, 2, -1)]
    # stage 2: receives all three micro-batches first
    acts += [A(2, S.RECV_ACT, m, 1, -1) for m in range(M)]
    assert S.verify(acts, 3) > 0
    # FIFO mix-up detection: micro-batches received in the wrong order
    bad = [A(0, S.FWD, 0, -1, -1), A(0, S.SEND_ACT, 0, 1, -1), A(0, S.FWD, 1, -1, -1),
           A(0, S.SEND_ACT, 1, 1, -1), A(1, S.RECV_ACT, 1, 0, -1), A(1, S.RECV_ACT, 0, 0, -1)]
    assert S.verify(bad, 2) < 0


def _ref_grads(seed, x):
    torch.manual_seed(seed)
    model = LLama(**TINY)
    loss = causalLLMLoss(model(x), x)
    loss.backward()
    return loss.item(), {n: p.grad.clone() for n, p in model.named_parameters()}


def _pp_worker(rank, world, port, kind, out_dir, micro, use_links=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ddl25spring_amd.parallel.pipeline import PipelineStage, pipeline_links
    links = pipeline_links(1, world) if use_links else None
    torch.manual_seed(0)
    model = LLama(**TINY)
    names = {id(p): n for n, p in model.named_parameters()}
    stage_mod = split_stages(model, world)[rank]
    torch.manual_seed(123)
    x = torch.randint(0, TINY["vocab_size"], (6, TINY["ctx_size"]))
    mbs = list(torch.chunk(x, micro))
    ps = PipelineStage(stage_mod, rank, world, act_shape=(6 // micro, TINY["ctx_size"], TINY["dmodel"]),
                       act_dtype=torch.float32, device=torch.device("cpu"), links=links)
    loss = ps.run(kind, micro, inputs=mbs, targets=mbs, loss_fn=lambda o, t: causalLLMLoss(o, t))
    grads = {names[id(p)]: p.grad.clone() for p in stage_mod.parameters() if p.grad is not None}
    torch.save({"loss": None if loss is None else loss.item(), "grads": grads},
               os.path.join(out_dir, f"r{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("kind,world,micro,use_links", [("gpipe", 3, 3, False), ("1f1b", 3, 3, False),
                                                        ("1f1b", 2, 6, False), ("naive", 2, 1, False),
                                                        ("1f1b", 3, 3, True), ("gpipe", 3, 3, True),
                                                        ("1f1b", 2, 6, True), ("naive", 3, 2, True)])
def test_pipeline_matches_single_process(kind, world, micro, use_links):
    """Blocking grouped P2P and the asynchronous per-link executor (receives posted before the
    preceding compute step) both reproduce the single-process gradients."""
    torch.manual_seed(123)
    x = torch.randint(0, TINY["vocab_size"], (6, TINY["ctx_size"]))
    # full-batch reference equals mean of micro-batch losses when micro-batches are equal-sized
    torch.manual_seed(0)
    model = LLama(**TINY)
    loss_ref = sum(causalLLMLoss(model(m), m) for m in torch.chunk(x, micro)) / micro
    loss_ref.backward()
    ref = {n: p.grad for n, p in model.named_parameters()}
    with tempfile.TemporaryDirectory() as d:
        port = 29700 + hash((kind, world, micro, use_links)) % 200
        mp.spawn(_pp_worker, args=(world, port, kind, d, micro, use_links), nprocs=world, join=True)
        res = [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True) for r in range(world)]
    assert abs(res[-1]["loss"] - loss_ref.item()) < 1e-5
    seen = set()
    for r in res:
        for n, g in r["grads"].items():
            assert torch.allclose(g, ref[n], atol=1e-5, rtol=1e-4), n
            seen.add(n)
    assert seen == set(ref)


def _dp_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    from ddl25spring_amd.parallel.dp import GradBucketer, broadcast_parameters
    from ddl25spring_amd.runtime import dist as rdist
    ctx = rdist.init(backend="gloo", device="cpu")
    torch.manual_seed(rank)  # different init on purpose: broadcast must fix it
    model = LLama(**TINY)
    broadcast_parameters(model, ctx)
    bk = GradBucketer(model, ctx, bucket_mb=0.01)  # many tiny buckets
    assert len(bk.buckets) > 3
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    torch.manual_seed(99)
    x = torch.randint(0, TINY["vocab_size"], (4, TINY["ctx_size"]))
    mine = x[rank * 2:(rank + 1) * 2]
    for _ in range(2):
        bk.zero_grad()
        causalLLMLoss(model(mine), mine).backward()
        bk.finish()
        opt.step()
    torch.save({n: p.detach().clone() for n, p in model.named_parameters()},
               os.path.join(out_dir, f"r{rank}.pt"))
    rdist.shutdown()


def test_data_parallel_ga_equals_large_batch():
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_dp_worker, args=(2, 29911, d), nprocs=2, join=True)
        w0 = torch.load(os.path.join(d, "r0.pt"), weights_only=True)
        w1 = torch.load(os.path.join(d, "r1.pt"), weights_only=True)
    torch.manual_seed(0)
    ref = LLama(**TINY)
    # rank 0's init was broadcast: rebuild it
    torch.manual_seed(0)
    ref = LLama(**TINY)
    opt = torch.optim.SGD(ref.parameters(), lr=0.1)
    torch.manual_seed(99)
    x = torch.randint(0, TINY["vocab_size"], (4, TINY["ctx_size"]))
    for _ in range(2):
        opt.zero_grad()
        loss = (causalLLMLoss(ref(x[:2]), x[:2]) + causalLLMLoss(ref(x[2:]), x[2:])) / 2
        loss.backward()
        opt.step()
    for n, p in ref.named_parameters():
        assert torch.equal(w0[n], w1[n]), n
        assert torch.allclose(w0[n], p.detach(), atol=1e-5), n


def _grid_worker(rank, world, port, out_dir, pp=2):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    from ddl25spring_amd.parallel.dp import GradBucketer
    from ddl25spring_amd.parallel.pipeline import PipelineStage, grid_ranks, pipeline_links
    from ddl25spring_amd.runtime import dist as rdist
    ctx = rdist.init(backend="gloo", device="cpu")
    dp = world // pp
    pipe, stage, pipe_ranks, dp_ranks = grid_ranks(rank, dp, pp)
    # collective creation of every DP group, in the same order on all ranks (fixes SURVEY Q2)
    dp_group = ctx.new_groups("dp", [[p * pp + s for p in range(dp)] for s in range(pp)])
    links = pipeline_links(dp, pp)  # collective: every rank, same order
    torch.manual_seed(0)
    model = LLama(**TINY)
    mod = split_stages(model, pp)[stage]
    bk = GradBucketer(mod, ctx, group=dp_group, bucket_mb=0.05)
    opt = torch.optim.Adam(mod.parameters(), lr=1e-3)
    torch.manual_seed(5)
    data = torch.randint(0, TINY["vocab_size"], (8, TINY["ctx_size"]))
    mine = data[pipe * 4:(pipe + 1) * 4]
    ps = PipelineStage(mod, stage, pp, ranks=pipe_ranks, act_shape=(2, TINY["ctx_size"], TINY["dmodel"]),
                       act_dtype=torch.float32, device=torch.device("cpu"), links=links)
    losses = []
    for it in range(3):
        bk.zero_grad()
        mbs = list(torch.chunk(mine, 2))
        loss = ps.run("1f1b", 2, inputs=mbs, targets=mbs, loss_fn=causalLLMLoss, grad_sync=bk)
        bk.finish()
        opt.step()
        if loss is not None:
            losses.append(loss.item())
    torch.save({"losses": losses, "w": [p.detach().clone() for p in mod.parameters()]},
               os.path.join(out_dir, f"r{rank}.pt"))
    rdist.shutdown()


@pytest.mark.parametrize("pp", [2, 3])
def test_dp_x_pp_grid_runs_and_replicas_agree(pp):
    """DP x PP grid, 1F1B with the asynchronous per-link P2P (one communicator per directed stage
    link, irecvs posted ahead) running beside the DP gradient bucketer's all-reduces on the DP
    groups: pp = 3 has a middle stage with two links in flight at once."""
    world = 2 * pp
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_grid_worker, args=(world, 29933 + pp, d, pp), nprocs=world, join=True)
        res = [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True) for r in range(world)]
    # stage s of pipeline 0 (rank s) and pipeline 1 (rank pp + s) hold identical weights
    for s in range(pp):
        for a, b in zip(res[s]["w"], res[pp + s]["w"]):
            assert torch.allclose(a, b, atol=1e-6)
    assert len(res[pp - 1]["losses"]) == 3 and len(res[2 * pp - 1]["losses"]) == 3


def _native_dp_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    import ddl25spring_amd.ops.reference as R
    from ddl25spring_amd.models import mnist_mlp
    from ddl25spring_amd.models import params as P
    from ddl25spring_amd.optim import SGD
    from ddl25spring_amd.parallel.dp import NativeGradBucketer
    from ddl25spring_amd.runtime import dist as rdist
    R._bf = lambda t: t.float()
    P.CPU_SHADOW_DTYPE = torch.float32
    ctx = rdist.init(backend="gloo", device="cpu")
    net = mnist_mlp().to("cpu", seed=rank)  # different init on purpose: the broadcast fixes it
    ctx.broadcast(net.store.data, 0)
    net.store.sync_shadow()
    bk = NativeGradBucketer(net, ctx, bucket_mb=0.05)  # several buckets
    assert len(bk.bounds) > 1
    net.grad_hook = bk.on_layer_done
    opt = SGD(net, lr=0.1)
    g = torch.Generator().manual_seed(7)
    x = torch.randn(1, 8, 800, generator=g)
    y = torch.randint(0, 10, (1, 8), generator=g, dtype=torch.int32)
    for _ in range(2):
        opt.zero_grad()
        net.train_step(x[:, rank * 4:(rank + 1) * 4], y[:, rank * 4:(rank + 1) * 4])
        bk.finish()
        opt.step()
    torch.save(net.store.data.clone(), os.path.join(out_dir, f"r{rank}.pt"))
    rdist.shutdown()


def test_native_dp_bucketer_equals_large_batch(monkeypatch):
    import ddl25spring_amd.ops.reference as R
    from ddl25spring_amd.models import mnist_mlp
    from ddl25spring_amd.models import params as P
    from ddl25spring_amd.optim import SGD
    monkeypatch.setattr(R, "_bf", lambda t: t.float())
    monkeypatch.setattr(P, "CPU_SHADOW_DTYPE", torch.float32)
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_native_dp_worker, args=(2, 29955, d), nprocs=2, join=True)
        w0 = torch.load(os.path.join(d, "r0.pt"), weights_only=True)
        w1 = torch.load(os.path.join(d, "r1.pt"), weights_only=True)
    net = mnist_mlp().to("cpu", seed=0)
    opt = SGD(net, lr=0.1)
    g = torch.Generator().manual_seed(7)
    x = torch.randn(1, 8, 800, generator=g)
    y = torch.randint(0, 10, (1, 8), generator=g, dtype=torch.int32)
    for _ in range(2):
        opt.zero_grad()
        net.train_step(x, y)
        opt.step()
    assert torch.equal(w0, w1)
    assert torch.allclose(w0, net.store.data, atol=1e-5)


def _flat_bucket_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    from ddl25spring_amd.optim import FlatAdam
    from ddl25spring_amd.parallel.dp import GradBucketer
    from ddl25spring_amd.runtime import dist as rdist
    ctx = rdist.init(backend="gloo", device="cpu")
    res = {}
    for mode in ("own", "flat"):
        torch.manual_seed(0)
        model = LLama(**TINY)
        opt = FlatAdam(model.parameters(), lr=1e-3)
        bk = GradBucketer(model, ctx, bucket_mb=0.02, flat=opt if mode == "flat" else None)
        torch.manual_seed(7 + rank)
        x = torch.randint(0, TINY["vocab_size"], (2, TINY["ctx_size"]))
        for _ in range(2):
            bk.zero_grad()  # (FlatAdam.zero_grad would re-point the grads away from own buckets)
            causalLLMLoss(model(x), x).backward()
            bk.finish()
            opt.step()
        res[mode] = opt.data.clone()
        if mode == "flat":  # the buckets ARE the optimizer's gradient buffer
            assert all(b["flat"].data_ptr() >= opt.grad.data_ptr() for b in bk.buckets)
    torch.save(res, os.path.join(out_dir, f"r{rank}.pt"))
    rdist.shutdown()


def test_grad_bucketer_on_flatadam_buffer_equals_own_buckets():
    """DP-GA buckets as slices of FlatAdam's flat grad (no second buffer, no copy in step) give
    bit-identical steps to separate bucket buffers, and replicas agree."""
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_flat_bucket_worker, args=(2, 29961, d), nprocs=2, join=True)
        res = [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True) for r in range(2)]
    for r in range(2):
        assert torch.equal(res[r]["own"], res[r]["flat"])
    assert torch.equal(res[0]["flat"], res[1]["flat"])
