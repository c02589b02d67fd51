"""Times the fused classifier head (Fn.head_train) against the per-layer chain it replaces
(avgpool -> fc FWD -> CE -> bias sum -> fc WGRAD -> fc DGRAD -> pool backward + BN reduce) on
ResNet-18 CIFAR head shapes, 1 and 8 clients.  python scripts/head_bench.py"""
import torch

from ddl25spring_amd.ops import functional as Fn
from ddl25spring_amd.ops.functional import ConvGeom


def timed(fn, reps=20):
    """GPU time per call: ``reps`` calls captured in one HIP graph, replayed (no host overhead)."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        for _ in range(reps):
            fn()
    graph.replay()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(5):
        graph.replay()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / (5 * reps) * 1e3


def main():
    dev = torch.device("cuda")
    for G in (1, 8):
        N, H, W, C, Kp, ncls = 100, 4, 4, 512, 32, 10
        x = torch.randn(G, N, H, W, C, device=dev).relu().to(torch.bfloat16)
        c = torch.randn(G, N, H, W, C, device=dev).to(torch.bfloat16)
        w = (torch.randn(G, Kp, 1, 1, C, device=dev) * 0.05).to(torch.bfloat16)
        b = torch.zeros(G, Kp, device=dev)
        dw, db = torch.zeros(G, Kp, 1, 1, C, device=dev), torch.zeros(G, Kp, device=dev)
        mean, rstd = torch.zeros(G, C, device=dev), torch.ones(G, C, device=dev)
        labels = torch.randint(0, ncls, (G, N), dtype=torch.int32, device=dev)
        res = {}
        res["fused"] = timed(lambda: Fn.head_train(x, w, b, labels, ncls, 1.0 / N, dw, db, bn=(c, mean, rstd)))
        g = ConvGeom(G, N, 1, 1, C, Kp, 1, 1, 1, 0)

        def chain():
            p = Fn.avgpool_fwd(x)
            z = Fn.conv_fwd(p.reshape(G, N, 1, 1, C), w, g, bias=b)
            loss, dz, _ = Fn.cross_entropy(z.reshape(G, N, Kp), labels, ncls=ncls, scale=1.0 / N)
            Fn.channel_sum(dz, db)
            dz4 = dz.reshape(G, N, 1, 1, Kp)
            Fn.conv_wgrad(dz4, p.reshape(G, N, 1, 1, C), g, dw)
            dp = Fn.conv_dgrad(dz4, w, g)
            Fn.avgpool_bwd_bn(dp.reshape(G, N, C), x, (c, mean, rstd))
        res["per-layer chain"] = timed(chain)
        print(f"G={G}: " + ", ".join(f"{k} {v:.1f} us" for k, v in res.items()), flush=True)


if __name__ == "__main__":
    main()
