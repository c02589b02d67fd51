"""ResNet-50 (batch 256) stride-1 1x1 convs: our implicit-GEMM forward with its BN-statistics
epilogue vs hipBLASLt on the same plain GEMM (no epilogue).  PYTHONPATH=. python scripts/r50_1x1_sol.py"""
import torch

from ddl25spring_amd.ops import functional as Fn
from ddl25spring_amd.ops.functional import ConvGeom
from scripts.conv_gemm_sol import timed  # noqa: E402


def main():
    dev = torch.device("cuda")
    N = 256
    for H, C, K in [(56, 64, 256), (56, 256, 64), (28, 128, 512), (28, 512, 128), (14, 256, 1024),
                    (14, 1024, 256), (7, 512, 2048), (7, 2048, 512)]:
        g = ConvGeom(1, N, H, H, C, K, 1, 1, 1, 0)
        M = N * H * H
        a = torch.randn(M, C, device=dev).to(torch.bfloat16)
        b = torch.randn(C, K, device=dev).to(torch.bfloat16)
        x = a.view(1, N, H, H, C)
        w = (torch.randn(1, K, 1, 1, C, device=dev) * 0.05).to(torch.bfloat16)
        st = Fn.stats_buffer(1, K, dev)
        fl = 2 * M * C * K
        t_b = timed(lambda: torch.matmul(a, b))
        t_o = timed(lambda: Fn.conv_fwd(x, w, g, stats=st))
        print(f"{H}x{H} {C}->{K}: M={M} ({fl / 1e9:.1f} GF): hipBLASLt {t_b:.1f} us ({fl / t_b / 1e6:.0f} TF), "
              f"ours + BN stats {t_o:.1f} us ({fl / t_o / 1e6:.0f} TF)", flush=True)


if __name__ == "__main__":
    main()
