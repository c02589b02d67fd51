"""Collective code paths on the one-GPU test box.

* RCCL: a world-1 ``nccl`` process group (``DDL_FORCE_PG=1``) runs ``init_process_group(device_id=)``,
  ``barrier(device_ids=)``, device-side scalar reductions, device all-reduce, the native and torch
  gradient bucketers' all-reduce hooks and the FL aggregation on real hardware (RCCL refuses two
  ranks on one GPU, so world > 1 over RCCL is the driver's 8-GPU job).
* Pipeline parallelism with device (bf16) activations: 3 gloo ranks share the GPU, each one stage of
  the LLaMA (reference lab/tutorial_1b/PP/1F1B/intro_PP_1F1B_MB.py:51-137), GPipe and 1F1B,
  against the unsplit single-process model.
"""
import json
import os
import subprocess
import sys
import tempfile

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_RCCL_SCRIPT = r"""
import json, torch, torch.distributed as dist
from ddl25spring_amd.runtime import dist as rdist
from ddl25spring_amd.parallel.dp import GradBucketer, NativeGradBucketer
ctx = rdist.init()
out = {"backend": dist.get_backend(), "distributed": ctx.is_distributed, "world": dist.get_world_size()}
ctx.barrier()
out["max"] = ctx.max_scalar(3.5)
t = torch.arange(1000, dtype=torch.float32, device=ctx.device)
ctx.all_reduce(t)
out["allreduce_ok"] = bool(torch.equal(t, torch.arange(1000, dtype=torch.float32, device=ctx.device)))
# native bucketer hooks on a ResNet-18 training step (fp32): grads unchanged by a world-1 all-reduce
from ddl25spring_amd.models import resnet18_cifar
from ddl25spring_amd.data.images import DeviceImageDataset, synthetic_images
net = resnet18_cifar(groups=1, precision="fp32").to(ctx.device, seed=3)
data = DeviceImageDataset(synthetic_images("cifar10", 64, seed=0), ctx.device, net.input_spec)
x, y = data.batch(torch.arange(32, dtype=torch.int32, device=ctx.device).view(1, 32))
net.store.grad.zero_(); net.train_step(x, y); ref = net.store.grad.clone()
b = NativeGradBucketer(net, ctx, bucket_mb=4.0)
net.grad_hook = b.on_layer_done
net.store.grad.zero_(); net.train_step(x, y); b.finish(); torch.cuda.synchronize()
out["native_buckets"] = len(b.bounds)
out["native_equal"] = bool(torch.equal(ref, net.store.grad))
# torch-module bucketer (LLaMA stage, bf16 device activations)
from ddl25spring_amd.models.llama import LLama, causalLLMLoss
torch.manual_seed(0)
m = LLama(vocab_size=512, dmodel=96, num_heads=3, n_layers=2, ctx_size=64).to(ctx.device)
tok = torch.randint(0, 512, (4, 64), device=ctx.device)
causalLLMLoss(m(tok), tok).backward()
ref = [p.grad.clone() for p in m.parameters()]
for p in m.parameters(): p.grad = None
gb = GradBucketer(m, ctx, bucket_mb=0.5)
gb.zero_grad(); causalLLMLoss(m(tok), tok).backward(); gb.finish(); torch.cuda.synchronize()
out["torch_buckets"] = len(gb.buckets)
out["torch_equal"] = all(torch.allclose(a, p.grad, rtol=1e-4, atol=1e-6) for a, p in zip(ref, m.parameters()))
print("RCCL_RESULT " + json.dumps(out))
rdist.shutdown()
"""


def _env(port):
    env = dict(os.environ, DDL_FORCE_PG="1", RANK="0", WORLD_SIZE="1", LOCAL_RANK="0",
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), PYTHONPATH=ROOT)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return env


def test_rccl_world1_collectives_and_bucketers(cuda):
    r = subprocess.run([sys.executable, "-c", _RCCL_SCRIPT], capture_output=True, text=True, timeout=600,
                       cwd=ROOT, env=_env(29811))
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("RCCL_RESULT ")]
    assert line, r.stdout[-2000:]
    out = json.loads(line[0].split(" ", 1)[1])
    assert out["backend"] == "nccl" and out["distributed"] and out["world"] == 1, out
    assert out["max"] == 3.5 and out["allreduce_ok"], out
    assert out["native_buckets"] >= 2 and out["native_equal"], out
    assert out["torch_buckets"] >= 2 and out["torch_equal"], out


def test_bench_over_world1_rccl(cuda):
    """bench.py with its collectives on RCCL (world-1 nccl group): aggregation all-reduce, device
    barrier and max-over-ranks timing all go through RCCL."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "1", "--warmup", "1",
                        "--train-size", "4000"], capture_output=True, text=True, timeout=600, cwd=ROOT,
                       env=_env(29812))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1 and json.loads(lines[0])["dtype"] == "fp32", r.stdout[-2000:]


def _pp_worker(rank, world, port, schedule, out, precision):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0")
    from ddl25spring_amd.apps.llm import LLMConfig, train_llm
    from ddl25spring_amd.runtime import dist as rdist
    ctx = rdist.init(backend="gloo", device="cuda")
    cfg = LLMConfig(vocab_size=512, dmodel=96, num_heads=3, n_layers=3, ctx_size=64, batch_size=3,
                    micro_batches=3, pp=world, schedule=schedule, iters=4, log_every=1, precision=precision)
    res = train_llm(cfg, ctx, log=None)
    if rank == world - 1:
        torch.save(torch.tensor([l for _, l in res["losses"]]), os.path.join(out, "pp.pt"))
    rdist.shutdown()


@pytest.mark.parametrize("schedule,precision", [("gpipe", "fp32"), ("1f1b", "fp32"), ("1f1b", "bf16")])
def test_pipeline_three_stages_device_activations_match_single_process(cuda, schedule, precision):
    """fp32 (the reference's precision: fp32 stage messages, deterministic kernels, asynchronous
    per-link P2P) matches the unsplit model to rounding; bf16 to bf16 tolerance."""
    from ddl25spring_amd.apps.llm import LLMConfig, train_llm
    from ddl25spring_amd.runtime.dist import DistContext
    cfg = LLMConfig(vocab_size=512, dmodel=96, num_heads=3, n_layers=3, ctx_size=64, batch_size=3,
                    micro_batches=3, pp=1, iters=4, log_every=1, graph=False, precision=precision)
    single = torch.tensor([l for _, l in train_llm(cfg, DistContext(device=cuda), log=None)["losses"]])
    port = 29821 + ["gpipe", "1f1b"].index(schedule) + 2 * (precision == "bf16")
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_pp_worker, args=(3, port, schedule, d, precision), nprocs=3, join=True)
        pp = torch.load(os.path.join(d, "pp.pt"), weights_only=True)
    assert pp.shape == single.shape and torch.isfinite(pp).all()
    tol = 1e-5 if precision == "fp32" else 2e-2
    assert torch.allclose(pp, single, rtol=tol, atol=tol), (pp, single)
