"""Speed-of-light check for the conv kernels: hipBLASLt (torch.matmul) on the plain GEMM each
ResNet-18 conv layer reduces to (im2col'd, no gather, no epilogue), 8 clients x batch 100, vs our
implicit-GEMM forward with its BN-statistics epilogue.  PYTHONPATH=. python scripts/conv_gemm_sol.py"""
import torch

from ddl25spring_amd.ops import functional as Fn
from ddl25spring_amd.ops.functional import ConvGeom


def timed(fn, reps=10):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(3):
        g.replay()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / (3 * reps) * 1e3


def main():
    dev = torch.device("cuda")
    G, N = 8, 100
    for name, (H, C, K) in {"c64": (32, 64, 64), "c128": (16, 128, 128), "c256": (8, 256, 256),
                            "c512": (4, 512, 512)}.items():
        g = ConvGeom(G, N, H, H, C, K, 3, 3, 1, 1)
        M, Kr = G * N * H * H, 9 * C
        a = torch.randn(M, Kr, device=dev).to(torch.bfloat16)
        b = torch.randn(Kr, K, device=dev).to(torch.bfloat16)
        x = torch.randn(G, N, H, H, C, device=dev).to(torch.bfloat16)
        w = (torch.randn(G, K, 3, 3, C, device=dev) * 0.05).to(torch.bfloat16)
        st = Fn.stats_buffer(G, K, dev)
        fl = 2 * M * Kr * K
        t_b = timed(lambda: torch.matmul(a, b))
        t_o = timed(lambda: Fn.conv_fwd(x, w, g, stats=st))
        print(f"{name}: GEMM {M}x{Kr}x{K} ({fl / 1e9:.1f} GF): hipBLASLt {t_b:.1f} us ({fl / t_b / 1e6:.0f} TF), "
              f"ours conv fwd + BN stats {t_o:.1f} us ({fl / t_o / 1e6:.0f} TF)", flush=True)


if __name__ == "__main__":
    main()
