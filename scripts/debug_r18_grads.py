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
ap.add_argument("--groups", type=int, default=2)
ap.add_argument("--batch", type=int, default=16)
ap.add_argument("--target-wg", type=int, default=0)
ap.add_argument("--quiet", action="store_true", help="only the worst error and the BAD parameters")
a = ap.parse_args()
if a.target_wg:
    F32.TARGET_WG = a.target_wg
F32.set_math(a.math)
F32.set_halo(bool(a.halo))
cuda = torch.device("cuda")
G = a.groups
tm, net, mapping, convert = _resnet_pair(cuda, G=G)
torch.manual_seed(1)
x = torch.randn(a.batch, 3, 32, 32)
y = torch.randint(0, 10, (a.batch,))
net.store.zero_grad()
xin = net.prepare_input(x.to(cuda))
loss, _ = net.train_step(torch.cat([xin] * G), torch.stack([y] * G).to(cuda, torch.int32))
import copy  # noqa: E402
t32 = copy.deepcopy(tm).float().to(cuda)  # stock torch fp32 (MIOpen) on the same GPU, for scale
F.cross_entropy(t32(x.to(cuda)), y.to(cuda)).backward()
t64 = tm.double()
lt = F.cross_entropy(t64(x.double()), y)
lt.backward()
g32 = {n: p.grad for n, p in t32.named_parameters()}
e32 = sorted(_err(g32[n], p.grad) for n, p in t64.named_parameters())
w32 = e32[-1]
print(f"stock torch fp32: worst relative gradient error {w32:.2e}, median {e32[len(e32) // 2]:.2e}")
print(f"G={G} B={a.batch} twg={a.target_wg} halo={a.halo} math={a.math} loss {loss[0].item():.8f} "
      f"ref {lt.item():.8f}")
for grp in range(G):
    g = convert.export_torch(net, t64, mapping, group=grp, grads=True)
    worst, bad, errs = 0.0, [], []
    for name, p in t64.named_parameters():
        e = _err(g[name], p.grad)
        errs.append(e)
        worst = max(worst, e)
        if e > 1e-4:
            bad.append(f"{name}:{e:.1e}")
        if not a.quiet:
            print(f"  {name:40s} {e:.2e} {'BAD' if e > 1e-4 else ''}")
    errs.sort()
    print(f"  group {grp}: worst {worst:.2e}, median {errs[len(errs) // 2]:.2e}; {len(bad)} bad: {' '.join(bad[:12])}")
