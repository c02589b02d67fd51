"""bf16 LLaMA HIP ops (linear / rmsnorm / swiglu / embedding / fused RoPE attention / vocab CE) vs
the fp32 PyTorch reference of the same op, and a whole-model fwd+bwd check. The device inputs are
bf16: the activation dtype selects the kernels, fp32 activations run the reference-precision path
(tests/test_llama_f32_gpu.py)."""
import pytest
import torch

from ddl25spring_amd.models.llama import LLama, causalLLMLoss
from ddl25spring_amd.ops import autograd_ops as A

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


BF = torch.bfloat16


def _pair(t, cuda, dtype=torch.float32):
    c = t.detach().clone().to(cuda, dtype).requires_grad_(True)
    h = t.detach().clone().float().requires_grad_(True)
    return c, h


@pytest.mark.parametrize("T,D", [(2048, 288), (4096, 288), (3, 2048), (1000, 520)])
def test_rmsnorm_backward_shapes(cuda, T, D):
    """Register-accumulated d(gamma): the LLaMA shape (8 x 256 tokens, 288 dims), more rows than the
    grid covers in one sweep, the widest supported D (all 4 lane chunks) and a partly filled chunk."""
    torch.manual_seed(1)
    x = torch.randn(T, D)
    gam = torch.rand(D) + 0.5
    xc, xh = _pair(x, cuda, BF); gc, gh = _pair(gam, cuda)
    yc, yh = A.rmsnorm(xc, gc), A.rmsnorm(xh, gh)
    assert _rel(yc, yh) < 1e-2
    g = torch.randn_like(yh)
    yc.backward(g.to(cuda)); yh.backward(g)
    assert _rel(xc.grad, xh.grad) < 2e-2
    assert _rel(gc.grad, gh.grad) < 1e-2


def test_rmsnorm_fork_sums_residual_gradient(cuda):
    """rmsnorm_fork(x) = (rmsnorm(x), x): the residual branch's gradient is added inside the HIP
    backward; compare with the fp32 op where autograd sums the two paths."""
    torch.manual_seed(2)
    x = torch.randn(4, 64, 288)
    gam = torch.rand(288) + 0.5
    w = torch.randn(288, 288) * 0.05
    xc, xh = _pair(x, cuda, BF); gc, gh = _pair(gam, cuda)
    hc, rc = A.rmsnorm_fork(xc, gc)
    hh, rh = A.rmsnorm_fork(xh, gh)
    assert _rel(rc, xh) < 1e-2
    yc = A.linear(hc, w.to(cuda), residual=rc)
    yh = hh @ w.t() + rh
    g = torch.randn_like(yh)
    yc.backward(g.to(cuda)); yh.backward(g)
    assert _rel(xc.grad, xh.grad) < 2e-2 and _rel(gc.grad, gh.grad) < 2e-2
    # residual output unused: the fork's second gradient is None
    xc2 = x.detach().clone().to(cuda, BF).requires_grad_(True)
    h2, _ = A.rmsnorm_fork(xc2, gc.detach())
    h2.float().sum().backward()
    xr = x.detach().clone().requires_grad_(True)
    A.rmsnorm(xr, gam).sum().backward()
    assert _rel(xc2.grad, xr.grad) < 2e-2


def test_linear_rmsnorm_swiglu_embedding(cuda):
    torch.manual_seed(0)
    x = torch.randn(2, 37, 96)
    w = torch.randn(160, 96) * 0.1
    b = torch.randn(160)
    r = torch.randn(2, 37, 160)
    xc, xh = _pair(x, cuda, BF); wc, wh = _pair(w, cuda); bc, bh = _pair(b, cuda); rc, rh = _pair(r, cuda, BF)
    yc = A.linear(xc, wc, bc, residual=rc)
    yh = A.linear(xh, wh, bh, residual=rh)
    assert _rel(yc, yh) < 1e-2
    g = torch.randn_like(yh)
    yc.backward(g.to(cuda)); yh.backward(g)
    for a_, b_ in ((xc, xh), (wc, wh), (bc, bh), (rc, rh)):
        assert _rel(a_.grad, b_.grad) < 2e-2
    # rmsnorm
    gam = torch.rand(96) + 0.5
    xc, xh = _pair(x, cuda, BF); gc, gh = _pair(gam, cuda)
    yc, yh = A.rmsnorm(xc, gc), A.rmsnorm(xh, gh)
    assert _rel(yc, yh) < 1e-2
    g = torch.randn_like(yh)
    yc.backward(g.to(cuda)); yh.backward(g)
    assert _rel(xc.grad, xh.grad) < 2e-2 and _rel(gc.grad, gh.grad) < 2e-2
    # swiglu
    ab = torch.randn(2, 37, 128)
    ac, ah = _pair(ab, cuda, BF)
    yc, yh = A.swiglu(ac), A.swiglu(ah)
    assert _rel(yc, yh) < 1e-2
    g = torch.randn_like(yh)
    yc.backward(g.to(cuda)); yh.backward(g)
    assert _rel(ac.grad, ah.grad) < 2e-2
    # embedding (padding row gets no grad)
    emb = torch.randn(50, 64)
    idx = torch.randint(0, 50, (3, 11)); idx[0, 0] = 0
    ec, eh = _pair(emb, cuda)
    yc, yh = A.embedding(idx.to(cuda), ec, 0), A.embedding(idx, eh, 0)
    assert _rel(yc, yh) < 1e-2
    g = torch.randn_like(yh)
    yc.backward(g.to(cuda)); yh.backward(g)
    assert _rel(ec.grad, eh.grad) < 1e-2 and ec.grad[0].abs().max() == 0


@pytest.mark.parametrize("B,S,H,hd", [(2, 256, 6, 48), (1, 100, 2, 64), (3, 64, 4, 32), (1, 77, 2, 128),
                                      (4, 256, 2, 48), (8, 130, 2, 32)])
def test_fused_rope_attention(cuda, B, S, H, hd):
    torch.manual_seed(1)
    qkv = torch.randn(B, S, 3 * H * hd)
    qc, qh = _pair(qkv, cuda, BF)
    oc = A.causal_attention(qc, H, hd)
    oh = A.causal_attention(qh, H, hd)
    assert _rel(oc, oh) < 1e-2
    g = torch.randn_like(oh)
    oc.backward(g.to(cuda)); oh.backward(g)
    for part in range(3):
        sl = slice(part * H * hd, (part + 1) * H * hd)
        assert _rel(qc.grad[..., sl], qh.grad[..., sl]) < 2e-2, part


def test_vocab_cross_entropy(cuda):
    torch.manual_seed(2)
    logits = torch.randn(3, 17, 32000) * 2
    tgt = torch.randint(0, 32000, (3, 17))
    tgt[0, 3] = -100
    lc, lh = _pair(logits, cuda, BF)
    a = A.cross_entropy_vocab(lc, tgt.to(cuda))
    b = A.cross_entropy_vocab(lh, tgt)
    assert abs(a.item() - b.item()) < 2e-2
    a.backward(); b.backward()
    assert _rel(lc.grad, lh.grad) < 2e-2
    # non-unit upstream gradient (the gradient made in forward is rescaled on the device), and a
    # second backward through the same graph (recomputed, not rescaled twice)
    for t in (lc, lh):
        t.grad = None
    a = A.cross_entropy_vocab(lc, tgt.to(cuda))
    b = A.cross_entropy_vocab(lh, tgt)
    (a * 0.25).backward(retain_graph=True); (b * 0.25).backward(retain_graph=True)
    assert _rel(lc.grad, lh.grad) < 2e-2
    (a * 0.5).backward(); (b * 0.5).backward()
    assert _rel(lc.grad, lh.grad) < 2e-2
    # a constant factor folded into the kernel (scale=) == scaling the loss
    for t in (lc, lh):
        t.grad = None
    a = A.cross_entropy_vocab(lc, tgt.to(cuda), scale=0.25)
    b = A.cross_entropy_vocab(lh, tgt) * 0.25
    assert abs(a.item() - b.item()) < 1e-2
    a.backward(); b.backward()
    assert _rel(lc.grad, lh.grad) < 2e-2


def test_llama_model_fwd_bwd_matches_fp32(cuda):
    cfg = dict(vocab_size=512, dmodel=96, num_heads=2, n_layers=2, ctx_size=64)
    torch.manual_seed(0)
    mh = LLama(**cfg)
    torch.manual_seed(0)
    mc = LLama(**cfg, precision="bf16").to(cuda)
    x = torch.randint(0, 512, (2, 64))
    lh = causalLLMLoss(mh(x), x)
    lc = causalLLMLoss(mc(x.to(cuda)), x.to(cuda))
    assert abs(lh.item() - lc.item()) < 2e-2 * lh.item()
    lh.backward(); lc.backward()
    for (n, ph), (_, pc) in zip(mh.named_parameters(), mc.named_parameters()):
        assert _rel(pc.grad, ph.grad) < 5e-2, n


def test_fused_grad_accumulation_and_bf16_shadow(cuda):
    """FlatAdam(fused=True, bf16_shadow=True): weight grads accumulate straight into the flat grad
    buffer and the GEMMs read the optimizer-refreshed bf16 shadow; three steps of two
    micro-batches track the plain path (fresh grads + AccumulateGrad, per-forward casts)."""
    from ddl25spring_amd.optim import FlatAdam
    cfg = dict(vocab_size=512, dmodel=96, num_heads=2, n_layers=2, ctx_size=64)
    models, opts = [], []
    for fused in (False, True):
        torch.manual_seed(0)
        m = LLama(**cfg, precision="bf16").to(cuda)
        models.append(m)
        opts.append(FlatAdam(m.parameters(), lr=1e-3, fused=fused, bf16_shadow=fused))
    torch.manual_seed(1)
    xs = [torch.randint(0, 512, (4, 64), device=cuda) for _ in range(3)]
    for x in xs:
        for m, opt in zip(models, opts):
            opt.zero_grad()
            for mb in x.chunk(2):
                (causalLLMLoss(m(mb), mb) / 2).backward()
            opt.step()
    for (n, a), (_, b) in zip(models[0].named_parameters(), models[1].named_parameters()):
        assert _rel(b, a) < 1e-2, n
    # the shadow is the bf16 image of the updated weights
    assert _rel(opts[1].shadow.float(), opts[1].data) < 1e-2


def test_llm_step_graph_replay_matches_eager(cuda):
    """apps.llm: the whole dp=pp=1 step (4 micro-batches fwd+bwd, fused Adam with a device step
    counter) replayed from one HIP graph gives the eager loss curve."""
    from ddl25spring_amd.apps.llm import LLMConfig, train_llm
    from ddl25spring_amd.runtime.dist import DistContext
    curves = []
    for graph in (False, True):
        cfg = LLMConfig(vocab_size=1024, dmodel=96, num_heads=2, n_layers=2, ctx_size=64, batch_size=8,
                        micro_batches=4, iters=6, log_every=1, graph=graph, precision="bf16")
        out = train_llm(cfg, DistContext(device=cuda), log=None)
        curves.append([v for _, v in out["losses"]])
    assert len(curves[0]) == 6
    for a, b in zip(*curves):
        assert abs(a - b) < 2e-2 * abs(a), curves
    assert curves[1][-1] < curves[1][0]


@pytest.mark.parametrize("T,C,V", [(8192, 288, 32000), (300, 96, 520), (77, 32, 8)])
def test_wide_gemm_matches_fp32(cuda, T, C, V):
    """The LM-head GEMM (gemm_bf16.hip) vs an fp32 torch matmul of the same bf16 operands,
    including tile overhangs on both edges."""
    from ddl25spring_amd.ops import functional as Fn
    torch.manual_seed(3)
    x = torch.randn(T, C, device=cuda).to(torch.bfloat16)
    w = (torch.randn(V, C, device=cuda) * 0.05).to(torch.bfloat16)
    y = Fn.gemm_nt_bf16(x, w)
    ref = x.float() @ w.float().t()
    err = ((y.float() - ref).abs().max() / ref.abs().max()).item()
    assert err < 1e-2, err  # bf16 output rounding
    # a padded output row stride (a strided logits view)
    out = torch.full((T, V + 8), 7.0, device=cuda, dtype=torch.bfloat16)
    Fn.gemm_nt_bf16(x, w, out=out[:, :V])
    assert torch.equal(out[:, :V], y) and (out[:, V:] == 7.0).all()
