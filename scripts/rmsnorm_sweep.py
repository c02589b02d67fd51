"""RMSNorm backward grid sweep: rows per wave vs kernel time at the LLaMA-288d shape (8 x 256 tokens).

usage: python scripts/rmsnorm_sweep.py [T] [D]
Times ddl_rmsnorm_bwd alone (HIP events over 200 launches) for each rows-per-wave setting.
"""
import sys

import torch

from ddl25spring_amd.ops.autograd_ops import K, ptr, stream

T = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
D = int(sys.argv[2]) if len(sys.argv) > 2 else 288
dev = torch.device("cuda", 0)
x = torch.randn(T, D, device=dev).to(torch.bfloat16)
g = torch.rand(D, device=dev) + 0.5
dy = torch.randn(T, D, device=dev).to(torch.bfloat16)
rstd = torch.rsqrt(x.float().pow(2).mean(-1) + 1e-6).contiguous()
dx = torch.empty_like(x)
dg = torch.zeros(D, device=dev)
lib = K()
for rows in (1, 2, 4, 8, 16, 0):
    lib.ddl_rmsnorm_bwd_set_rows(rows)
    for _ in range(20):
        lib.ddl_rmsnorm_bwd(ptr(x), ptr(g), ptr(rstd), ptr(dy), None, ptr(dx), ptr(dg), T, D, stream())
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(200):
        lib.ddl_rmsnorm_bwd(ptr(x), ptr(g), ptr(rstd), ptr(dy), None, ptr(dx), ptr(dg), T, D, stream())
    e1.record()
    torch.cuda.synchronize()
    print(f"T={T} D={D} rows/wave={rows or 'auto'}: {e0.elapsed_time(e1) / 200 * 1000:.2f} us per launch", flush=True)
# numerics at the last setting vs fp32
dg.zero_()
lib.ddl_rmsnorm_bwd(ptr(x), ptr(g), ptr(rstd), ptr(dy), None, ptr(dx), ptr(dg), T, D, stream())
xf, dyf = x.float(), dy.float()
r = rstd[:, None]
dot = (g * dyf * xf).sum(-1, keepdim=True) / D
ref_dx = r * g * dyf - xf * r ** 3 * dot
ref_dg = (dyf * xf * r).sum(0)
print("rel dx", ((dx.float() - ref_dx).norm() / ref_dx.norm()).item(),
      "rel dg", ((dg - ref_dg).norm() / ref_dg.norm()).item())
