"""Per-parameter gradient error of one fp32 ResNet-18 step vs float64 torch, per engine setting.
    python scripts/debug_r18_grads.py [--halo 0|1] [--math x6]"""
import argparse
import sys
from pathlib import Path

import torch
import torch.nn.functional as F

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "tests"))
from ddl25spring_amd.ops import functional_f32 as F32  # noqa: E402
from test_fp32_gpu import _err, _resnet_pair  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--halo", type=int, default=1)
ap.add_argument("--math", default="x6")
a = ap.parse_args()
F32.set_math(a.math)
F32.set_halo(bool(a.halo))
cuda = torch.device("cuda")
tm, net, mapping, convert = _resnet_pair(cuda, G=2)
torch.manual_seed(1)
x = torch.randn(16, 3, 32, 32)
y = torch.randint(0, 10, (16,))
net.store.zero_grad()
xin = net.prepare_input(x.to(cuda))
loss, _ = net.train_step(torch.cat([xin, xin]), torch.stack([y, y]).to(cuda, torch.int32))
t64 = tm.double()
lt = F.cross_entropy(t64(x.double()), y)
lt.backward()
print(f"halo={a.halo} math={a.math} loss {loss[0].item():.8f} ref {lt.item():.8f}")
g = convert.export_torch(net, t64, mapping, group=0, grads=True)
for name, p in t64.named_parameters():
    e = _err(g[name], p.grad)
    print(f"  {name:40s} {e:.2e} {'BAD' if e > 1e-4 else ''}")
