"""X6 planes GEMM (csrc/kernels/gemm_x6.hip, ops/gemm_x6.py) against float64 torch: every operand
orientation, every tile / ring configuration, split-K, the residual / accumulate / bias epilogue,
tile overhang on every edge, exact planes and bitwise determinism; plus the fp32 linear layer on
each of its native engines (ops/llama_f32.py LINEAR)."""
import pytest
import torch

from ddl25spring_amd.ops import gemm_x6 as G

pytestmark = pytest.mark.gpu


def _rel_max(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).abs().max() / (b.abs().max() + 1e-30)).item()


def test_planes_exact(cuda):
    """h + m + l == x bitwise for |x| >= 2^-110 (below that the l / m pieces fall into the subnormal
    range, where the truncating split drops their last bits: a relative 2^-16..2^-24 of a value
    within 2^-110 of zero)."""
    torch.manual_seed(0)
    x = torch.randn(37, 56, device=cuda) * torch.logspace(-20, 20, 56, device=cuda)
    x[0, :8] = torch.tensor([0.0, -0.0, 1e-30, -1e-32, 3.4e38, -3.4e38, 1.0, -2.5])
    p = G.split(x)
    assert p.data.shape == (3, 64, 64)  # zero-padded to whole 32-deep stages
    assert p.data[:, 37:].abs().sum() == 0 and p.data[:, :, 56:].abs().sum() == 0
    assert torch.equal(p.dense(), x)


@pytest.mark.parametrize("plan", [(4, 4, 3, 1), (3, 4, 3, 1), (4, 2, 4, 1), (3, 2, 4, 1), (2, 4, 4, 1), (2, 2, 4, 1),
                                  (4, 4, 3, 3), (3, 2, 4, 5)])
@pytest.mark.parametrize("amn,bmn", [(False, False), (True, False), (False, True), (True, True)])
def test_gemm_orientations_plans(cuda, plan, amn, bmn):
    """out[q][p] = sum_k A(p, k) B(q, k) with overhanging tiles on M, N and K (M, N, K % 8 only)."""
    torch.manual_seed(1)
    M, N, K = 200, 136, 456
    A = torch.randn(K, M) if amn else torch.randn(M, K)
    B = torch.randn(K, N) if bmn else torch.randn(N, K)
    Ad = A.t() if amn else A
    Bd = B.t() if bmn else B
    ref = Bd.double() @ Ad.double().t()
    pa, pb = G.split(A.to(cuda)), G.split(B.to(cuda))
    out = torch.full((N, M), float("nan"), device=cuda)
    G._PLANS.clear()
    G._PLANS[(M, N, K)] = plan
    try:
        G.gemm(pa, amn, pb, bmn, out)
    finally:
        G._PLANS.clear()
    assert _rel_max(out, ref) < 2e-6


def test_gemm_epilogue_and_determinism(cuda):
    torch.manual_seed(2)
    M, N, K = 288, 512, 8192
    x, dy = torch.randn(K, M, device=cuda), torch.randn(K, N, device=cuda) * 0.01
    px, pd = G.split(x), G.split(dy)
    base = torch.randn(N, M, device=cuda)
    ref = dy.double().t() @ x.double()
    # WGRAD-style accumulate into an existing gradient (split-K by the default plan)
    out = base.clone()
    G.gemm(px, True, pd, True, out, accumulate=True)
    assert G.plan(M, N, K)[3] > 1  # the default plan splits this small-output, long-K product
    assert _rel_max(out, base.double().cpu() + ref.cpu()) < 2e-6
    out2 = base.clone()
    G.gemm(px, True, pd, True, out2, accumulate=True)
    assert torch.equal(out, out2)  # deterministic: slices folded in order, no atomics
    # residual + bias + alpha, unsplit
    res, bias = torch.randn(N, M, device=cuda), torch.randn(M, device=cuda)
    o3 = torch.empty(N, M, device=cuda)
    G.gemm(px, True, pd, True, o3, residual=res, bias=bias, alpha=0.5, split_k=1)
    want = 0.5 * ref + res.double() + bias.double().view(1, M)
    assert _rel_max(o3, want) < 2e-6
    # a row-strided output (ldo > M)
    big = torch.zeros(N, M + 64, device=cuda)
    G.gemm(px, True, pd, True, big[:, :M], split_k=1)
    assert _rel_max(big[:, :M], ref) < 2e-6 and big[:, M:].abs().max() == 0


@pytest.mark.parametrize("engine", ["x6g", "conv"])
@pytest.mark.parametrize("T,C,K,bias,res", [(256, 288, 864, False, True), (512, 768, 288, True, False),
                                            (128, 96, 160, False, False)])
def test_linear_f32_engines(cuda, engine, T, C, K, bias, res):
    """The fp32 linear on each native engine, FWD / DGRAD / WGRAD vs float64 (grad sink off)."""
    from ddl25spring_amd.ops import autograd_ops as A
    from ddl25spring_amd.ops import llama_f32 as L
    torch.manual_seed(3)
    x, w, b, r = torch.randn(T, C), torch.randn(K, C) * 0.05, torch.randn(K), torch.randn(T, K)
    mk = lambda t: (t.clone().to(cuda).requires_grad_(True), t.clone().double().requires_grad_(True))  # noqa: E731
    (xc, xh), (wc, wh), (bc, bh), (rc, rh) = mk(x), mk(w), mk(b), mk(r)
    old = L.LINEAR[0]
    L.LINEAR[0] = engine
    try:
        yc = A.linear(xc, wc, bc if bias else None, rc if res else None)
        g = torch.randn(T, K)
        yc.backward(g.to(cuda))
    finally:
        L.LINEAR[0] = old
    yh = A.linear(xh, wh, bh if bias else None, rh if res else None)
    yh.backward(g.double())
    assert _rel_max(yc, yh) < 2e-6
    assert _rel_max(xc.grad, xh.grad) < 2e-6 and _rel_max(wc.grad, wh.grad) < 2e-6
    if bias:
        assert _rel_max(bc.grad, bh.grad) < 2e-6
