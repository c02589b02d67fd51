"""Multi-rank FL on the device: 2 ranks share the one GPU of the test box over gloo (RCCL needs one
GPU per rank; the 8-GPU RCCL run is the driver's), exercising slot assignment, device-tensor
collectives and the replicated server state exactly as the 8-GPU bench does."""
import json
import os
import subprocess
import sys
import tempfile

import pytest
import torch
import torch.multiprocessing as mp

from ddl25spring_amd.data.images import DeviceImageDataset, synthetic_images
from ddl25spring_amd.data.split import split
from ddl25spring_amd.fl.algorithms import FedAvg
from ddl25spring_amd.models import mnist_mlp
from ddl25spring_amd.runtime.dist import DistContext

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from ddl25spring_amd.runtime import dist as rdist
    ctx = rdist.init(backend="gloo", device="cuda")
    arr = synthetic_images("mnist", 800, seed=0)
    parts = split(4, True, 1, labels=arr.labels)
    fa = FedAvg(mnist_mlp, DeviceImageDataset(arr, ctx.device), parts, lr=0.05, batch_size=50,
                client_fraction=1.0, seed=1, ctx=ctx, eval_every=0)
    fa.round()
    fa.round()
    torch.save(fa.w_global.cpu(), os.path.join(out, f"w{rank}.pt"))
    rdist.shutdown()


def test_two_ranks_one_gpu_match_single_process(cuda):
    arr = synthetic_images("mnist", 800, seed=0)
    parts = split(4, True, 1, labels=arr.labels)
    single = FedAvg(mnist_mlp, DeviceImageDataset(arr, cuda), parts, lr=0.05, batch_size=50,
                    client_fraction=1.0, seed=1, ctx=DistContext(device=cuda), eval_every=0)
    w0 = single.w_global.clone()
    single.round()
    single.round()
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(2, 29733, d), nprocs=2, join=True)
        ws = [torch.load(os.path.join(d, f"w{r}.pt"), weights_only=True) for r in range(2)]
    assert torch.equal(ws[0], ws[1])  # replicated server state
    upd = (single.w_global - w0).norm()
    assert ((ws[0].to(cuda) - single.w_global).norm() / upd).item() < 2e-2


def _worker_r18(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), DDL_F32_TARGET_WG="1",
                      DDL_F32_TUNED="0")
    from ddl25spring_amd.ops import functional_f32 as F32
    from ddl25spring_amd.runtime import dist as rdist
    # the module is already imported (the test module's imports): set the plan knobs directly
    F32.TARGET_WG, F32._TUNED = 1, {}
    F32._PLANS.clear()
    ctx = rdist.init(backend="gloo", device="cuda")
    fa = _r18_fedavg(ctx)
    fa.round()
    fa.round()
    torch.save(fa.w_global.cpu(), os.path.join(out, f"w{rank}.pt"))
    rdist.shutdown()


def _r18_fedavg(ctx):
    import functools
    from ddl25spring_amd.models import resnet18_cifar
    arr = synthetic_images("cifar10", 400, seed=0)
    parts = split(2, True, 1, labels=arr.labels)
    return FedAvg(functools.partial(resnet18_cifar, precision="fp32"), DeviceImageDataset(arr, ctx.device),
                  parts, lr=0.05, batch_size=50, client_fraction=1.0, seed=1, ctx=ctx, eval_every=0)


def test_fp32_resnet18_two_ranks_match_single_process(cuda):
    """The headline workload's multi-rank path at the reference's precision:
    2 gloo ranks share the GPU, one client slot each, vs one process holding both clients. With
    split-K pinned off and the tuned-plan table off (DDL_F32_TARGET_WG=1, DDL_F32_TUNED=0, so a
    client's kernels run the same tiles at G=1 and G=2) the only difference left is the aggregation's rounding (fused multiply-add over the
    process's clients vs a per-rank product then the all-reduce add): <= 1e-6 relative after two
    rounds, and both ranks hold the identical server model (same w_global sha256)."""
    import hashlib
    from ddl25spring_amd.ops import functional_f32 as F32
    old, old_tuned = F32.TARGET_WG, F32._TUNED
    F32.TARGET_WG, F32._TUNED = 1, {}
    F32._PLANS.clear()
    try:
        single = _r18_fedavg(DistContext(device=cuda))
        w0 = single.w_global.clone()
        single.round()
        single.round()
    finally:
        F32.TARGET_WG, F32._TUNED = old, old_tuned
        F32._PLANS.clear()
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker_r18, args=(2, 29737, d), nprocs=2, join=True)
        ws = [torch.load(os.path.join(d, f"w{r}.pt"), weights_only=True) for r in range(2)]
    shas = [hashlib.sha256(w.numpy().tobytes()).hexdigest() for w in ws]
    assert shas[0] == shas[1]
    ref = single.w_global.cpu()
    rel_w = ((ws[0] - ref).norm() / ref.norm()).item()
    rel_upd = ((ws[0] - ref).norm() / (ref - w0.cpu()).norm()).item()
    print(f"fp32 ResNet-18 2-rank vs 1-process: rel(w) {rel_w:.2e}, rel(update) {rel_upd:.2e}")
    assert rel_w <= 1e-6 and rel_upd < 1e-4, (rel_w, rel_upd)


def test_bench_two_ranks_gloo(cuda):
    """bench.py end to end with world 2 (the driver's torchrun path, gloo instead of RCCL)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", "29741", os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "1", "--warmup", "1", "--backend", "gloo", "--train-size", "8000"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1 and '"n_gpus": 2' in lines[0], out.stdout[-2000:]


def test_federated_gan_two_ranks_share_gpu(tmp_path):
    """Federated DCGAN with one client per rank on the device: 2 ranks share the
    GPU (auto gloo: more ranks than GPUs) and match the single-process run."""
    from ddl25spring_amd.runtime.launch import launch
    args = ["gan", "--clients", "2", "--rounds", "2", "--local-steps", "2", "--batch-size", "16",
            "--train-size", "128", "--seed", "3"]
    w1, w2 = tmp_path / "w1.pt", tmp_path / "w2.pt"
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    subprocess.run([sys.executable, "-m", "ddl25spring_amd", *args, "--save", str(w1)], check=True,
                   env=env, timeout=300, cwd=ROOT)
    res = launch([sys.executable, "-m", "ddl25spring_amd", *args, "--save", str(w2)], world=2,
                 log_dir=str(tmp_path / "logs"), timeout=300)
    assert res["returncode"] == 0, res
    a, b = torch.load(w1, weights_only=True), torch.load(w2, weights_only=True)
    assert a.shape == b.shape and torch.isfinite(b).all()
    # same clients, same data, same noise. One process batches both clients (groups=2), each rank
    # runs one (groups=1): different split-K / tile plans round the bf16 GEMMs differently, and 4
    # Adam steps amplify that to ~1e-3 of the weights (measured 1.3e-3); a wrong client->rank
    # assignment or noise stream gives O(1)
    assert ((a - b).norm() / a.norm()).item() < 1e-2


def test_vfl_gan_bench_two_ranks_share_gpu():
    """benchmarks/bench_vfl_gan.py at world 2: rank 0 = active party + GAN client 0, rank 1 =
    passive party + GAN client 1; cut-layer tensors host-staged over gloo."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", "29745",
           os.path.join(ROOT, "benchmarks", "bench_vfl_gan.py"), "--steps", "2", "--warmup", "1",
           "--local-steps", "4"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    # the split-NN + fp32 DCGAN line, then the labelled bf16 DCGAN line
    assert len(lines) == 2 and all('"n_gpus": 2' in l for l in lines), out.stdout[-2000:]
    assert json.loads(lines[0])["dtype"].endswith("fp32 (DCGAN)") and json.loads(lines[1])["dtype"] == "bf16"
    print(lines[0])


def _bench_json(stdout):
    import json
    lines = [l for l in stdout.splitlines() if l.startswith("{")]
    assert lines, stdout[-2000:]
    return json.loads(lines[0])


def test_bench_eight_ranks_one_slot_each_match_single_process():
    """The driver's 8-GPU headline layout rehearsed on one GPU: bench.py through torchrun with 8
    gloo ranks sharing the device, ONE client slot per rank (--clients = world), vs the
    single-process run holding all 8 clients as slots. Plans pinned so a client runs the same tiles
    at G = 1 and G = 8 (DDL_F32_TARGET_WG=1: no split-K; DDL_F32_TUNED=0). With the rank-ordered
    FedAvg mean (fl/aggregate.py) the 8-rank model is bitwise the single-process one, and every
    rank holds the same bits (rank_hashes_equal)."""
    env = dict(os.environ, DDL_F32_TARGET_WG="1", DDL_F32_TUNED="0", OMP_NUM_THREADS="2")
    common = [os.path.join(ROOT, "bench.py"), "--steps", "1", "--warmup", "1", "--clients", "8",
              "--train-size", "1600", "--deterministic"]
    one = subprocess.run([sys.executable, *common], capture_output=True, text=True, timeout=900, cwd=ROOT, env=env)
    assert one.returncode == 0, one.stderr[-3000:]
    eight = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=8",
                            "--master-addr", "127.0.0.1", "--master-port", "29751", *common, "--gpus", "8",
                            "--backend", "gloo"], capture_output=True, text=True, timeout=900, cwd=ROOT, env=env)
    assert eight.returncode == 0, eight.stderr[-3000:]
    a, b = _bench_json(one.stdout), _bench_json(eight.stdout)
    print(json.dumps({k: b[k] for k in ("n_gpus", "aggregation", "comm", "rank_hashes_equal", "value")}))
    assert b["n_gpus"] == 8 and b["config"]["client_slots_per_gpu"] == 1 and a["config"]["client_slots_per_gpu"] == 8
    assert b["rank_hashes_equal"] is True and b["aggregation"].startswith("rank-ordered")
    assert b["comm"]["transport"] == "all_gather"  # gloo: no IPC peer-read path
    assert a["w_global_sha256"] == b["w_global_sha256"]


def test_bench_eight_ranks_tuned_plans_rank_hashes_equal():
    """The same 8-rank rehearsal with the plans an 8-GPU run actually uses: the tuned plan table ON
    and split-K free (no DDL_F32_TUNED / DDL_F32_TARGET_WG pins), i.e. the G = 1 tuned entries. The
    model is then not bitwise the G = 8 single-process one (different tiles), but every rank must
    still hold the same bits after the rank-ordered FedAvg (rank_hashes_equal)."""
    env = dict(os.environ, OMP_NUM_THREADS="2")
    env.pop("DDL_F32_TUNED", None)
    env.pop("DDL_F32_TARGET_WG", None)
    common = [os.path.join(ROOT, "bench.py"), "--steps", "1", "--warmup", "1", "--clients", "8",
              "--train-size", "1600", "--deterministic"]
    eight = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=8",
                            "--master-addr", "127.0.0.1", "--master-port", "29753", *common, "--gpus", "8",
                            "--backend", "gloo"], capture_output=True, text=True, timeout=900, cwd=ROOT, env=env)
    assert eight.returncode == 0, eight.stderr[-3000:]
    b = _bench_json(eight.stdout)
    print(json.dumps({k: b[k] for k in ("n_gpus", "aggregation", "comm", "rank_hashes_equal", "value")}))
    assert b["n_gpus"] == 8 and b["config"]["client_slots_per_gpu"] == 1
    assert b["rank_hashes_equal"] is True
