"""Our MFMA linear (conv-GEMM family) vs torch.matmul (hipBLASLt) on the LLaMA-288 LM-head and
block shapes, graph-timed.  PYTHONPATH=. python scripts/gemm_vs_blas.py"""
import torch

from ddl25spring_amd.ops import functional as Fn


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
    for T, C, K in [(8192, 288, 32000), (8192, 288, 864), (8192, 768, 288), (8192, 288, 1536)]:
        x = torch.randn(T, C, device=dev).to(torch.bfloat16)
        w = (torch.randn(K, C, device=dev) * 0.05).to(torch.bfloat16)
        dy = torch.randn(T, K, device=dev).to(torch.bfloat16)
        g = Fn.ConvGeom(1, T, 1, 1, C, K, 1, 1, 1, 0)
        x5, w5, dy5 = x.view(1, T, 1, 1, C), w.view(1, K, 1, 1, C), dy.view(1, T, 1, 1, K)
        dw = torch.zeros(1, K, 1, 1, C, device=dev)
        fl = 2 * T * C * K
        r = {}
        r["ours fwd"] = timed(lambda: Fn.conv_fwd(x5, w5, g))
        r["blas fwd"] = timed(lambda: torch.matmul(x, w.t()))
        if Fn.gemm_nt_ok(C, K):
            r["ours wide fwd"] = timed(lambda: Fn.gemm_nt_bf16(x, w))
        r["ours dgrad+wgrad"] = timed(lambda: Fn.conv_dgrad_wgrad(dy5, w5, x5, g, dw))
        r["blas dx"] = timed(lambda: torch.matmul(dy, w))
        r["blas dw bf16"] = timed(lambda: torch.matmul(dy.t(), x))
        try:
            r["blas dw fp32-out"] = timed(lambda: torch.mm(dy.t(), x, out_dtype=torch.float32))
        except Exception as e:  # noqa: BLE001
            print("out_dtype unsupported:", type(e).__name__, str(e)[:80])
        print(f"T={T} C={C} K={K}: " + ", ".join(f"{k} {v:.1f} us ({fl / v / 1e6:.0f} TF)" for k, v in r.items()),
              flush=True)


if __name__ == "__main__":
    main()
