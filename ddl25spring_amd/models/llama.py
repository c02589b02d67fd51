"""Tiny LLaMA for the data/pipeline-parallel tutorials, with the reference's stage API.

The reference imports these from the external ``simplellm`` package (not vendored, not
installable here): ``LLama(CausalLLama, vocab, dmodel, num_heads, device, n_layers,
ctx_size, padding_idx)``, ``LLamaFirstStage(...).embed(x)``, ``LLamaStage``, ``LLamaLastStage``,
``causalLLMLoss`` (call sites lab/tutorial_1b/primer/intro.py:17-18,
PP/1F1B/intro_PP_1F1B.py:29-39,53,78-79). simplellm's internals are unverified, so the
architecture is the standard pre-norm LLaMA block: RMSNorm -> fused QKV -> causal attention with
interleaved RoPE -> out-proj (+residual, fused in the GEMM epilogue) -> RMSNorm -> fused [w1|w3]
SwiGLU FFN (hidden = 8/3 d rounded to 32) -> w2 (+residual) ; final RMSNorm and an untied LM head.
Loss-curve comparisons with the reference are therefore trend-level.

Precision (extension): ``precision="fp32"`` (default: the reference trains this model in fp32,
lab/tutorial_1b/PP/1F1B/intro_PP_1F1B_MB.py:16-46) makes the embedding emit fp32 activations, so
every op downstream runs the reference-precision kernels (ops/llama_f32.py: linears on the X6 /
exact-fp32 conv engine, fp32 attention / RMSNorm / SwiGLU / CE, all deterministic);
``precision="bf16"`` is the bf16-MFMA fast path. On CPU everything is fp32 either way.

Stage 0's ``embed`` runs the embedding AND the stage's blocks (the reference's rank 0 only calls
``embed``, so whether its blocks ran was simplellm-dependent).
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from ..ops import autograd_ops as A


def _ffn_hidden(d: int) -> int:
    return int(math.ceil(8 * d / 3 / 32) * 32)


class Block(nn.Module):
    def __init__(self, dmodel: int, num_heads: int, ffn_hidden: int | None = None):
        super().__init__()
        assert dmodel % num_heads == 0
        self.h, self.hd = num_heads, dmodel // num_heads
        F = ffn_hidden or _ffn_hidden(dmodel)
        self.norm1 = nn.Parameter(torch.ones(dmodel))
        self.norm2 = nn.Parameter(torch.ones(dmodel))
        self.wqkv = nn.Parameter(torch.empty(3 * dmodel, dmodel))
        self.wo = nn.Parameter(torch.empty(dmodel, dmodel))
        self.w13 = nn.Parameter(torch.empty(2 * F, dmodel))
        self.w2 = nn.Parameter(torch.empty(dmodel, F))
        for w in (self.wqkv, self.wo, self.w13, self.w2):
            nn.init.normal_(w, std=0.02)
        with torch.no_grad():
            self.wo.mul_(1 / math.sqrt(2))
            self.w2.mul_(1 / math.sqrt(2))

    def forward(self, x):  # x [B, S, D]
        h, x = A.rmsnorm_fork(x, self.norm1)
        qkv = A.linear(h, self.wqkv)
        att = A.causal_attention(qkv, self.h, self.hd)
        x = A.linear(att, self.wo, residual=x)
        h, x = A.rmsnorm_fork(x, self.norm2)
        return A.linear(A.swiglu(A.linear(h, self.w13)), self.w2, residual=x)


class CausalLLama:
    """Marker type, as passed to ``LLama(CausalLLama, ...)`` in the reference."""


PRECISIONS = ("fp32", "bf16")


def _act_dtype(precision: str):
    if precision not in PRECISIONS:
        raise ValueError(f"LLaMA precision must be one of {PRECISIONS}, got {precision!r}")
    return torch.float32 if precision == "fp32" else torch.bfloat16


class _Base(nn.Module):
    def __init__(self, dmodel, num_heads, n_layers, ctx_size, device=None, ffn_hidden=None, precision="fp32"):
        super().__init__()
        self.dmodel, self.ctx_size = dmodel, ctx_size
        self.precision = precision
        self.act_dtype = _act_dtype(precision)
        self.layers = nn.ModuleList(Block(dmodel, num_heads, ffn_hidden) for _ in range(n_layers))
        if device is not None:
            self.to(device)

    def run_layers(self, x):
        for blk in self.layers:
            x = blk(x)
        return x


class LLamaFirstStage(_Base):
    def __init__(self, vocab_size, dmodel=288, num_heads=6, device=None, n_layers=2, ctx_size=256,
                 padding_idx=None, ffn_hidden=None, precision="fp32"):
        super().__init__(dmodel, num_heads, n_layers, ctx_size, None, ffn_hidden, precision)
        self.vocab_size, self.padding_idx = vocab_size, padding_idx
        self.emb = nn.Parameter(torch.randn(vocab_size, dmodel) * 0.02)
        if device is not None:
            self.to(device)

    def embed(self, x):
        return self.run_layers(A.embedding(x, self.emb, self.padding_idx, dtype=self.act_dtype))

    forward = embed


class LLamaStage(_Base):
    def __init__(self, dmodel=288, num_heads=6, device=None, n_layers=2, ctx_size=256, ffn_hidden=None,
                 precision="fp32"):
        super().__init__(dmodel, num_heads, n_layers, ctx_size, device, ffn_hidden, precision)

    def forward(self, x):
        return self.run_layers(x)


class LLamaLastStage(_Base):
    def __init__(self, vocab_size, dmodel=288, num_heads=6, device=None, n_layers=2, ctx_size=256,
                 ffn_hidden=None, precision="fp32"):
        super().__init__(dmodel, num_heads, n_layers, ctx_size, None, ffn_hidden, precision)
        self.vocab_size = vocab_size
        self.norm = nn.Parameter(torch.ones(dmodel))
        self.head = nn.Parameter(torch.randn(vocab_size, dmodel) * 0.02)
        if device is not None:
            self.to(device)

    def forward(self, x):
        return A.linear(A.rmsnorm(self.run_layers(x), self.norm), self.head)


class LLama(nn.Module):
    """Whole model (reference primer/intro.py:17-18): first stage + last stage, n_layers total."""

    def __init__(self, kind=CausalLLama, vocab_size=32000, dmodel=288, num_heads=6, device=None,
                 n_layers=6, ctx_size=256, padding_idx=None, ffn_hidden=None, precision="fp32"):
        super().__init__()
        n0 = n_layers // 2
        self.precision = precision
        self.first = LLamaFirstStage(vocab_size, dmodel, num_heads, None, n0, ctx_size, padding_idx,
                                     ffn_hidden, precision)
        self.last = LLamaLastStage(vocab_size, dmodel, num_heads, None, n_layers - n0, ctx_size, ffn_hidden,
                                   precision)
        if device is not None:
            self.to(device)

    def forward(self, x):
        return self.last(self.first.embed(x))


def split_stages(model: LLama, n_stages: int):
    """Cut a whole LLama into n_stages modules sharing its parameters (first / middle / last)."""
    blocks = list(model.first.layers) + list(model.last.layers)
    per = [len(blocks) // n_stages + (1 if i < len(blocks) % n_stages else 0) for i in range(n_stages)]
    out, s = [], 0
    for i, n in enumerate(per):
        mine = blocks[s:s + n]
        s += n
        if i == 0:
            st = LLamaFirstStage.__new__(LLamaFirstStage)
            nn.Module.__init__(st)
            st.emb, st.padding_idx, st.vocab_size = model.first.emb, model.first.padding_idx, model.first.vocab_size
        elif i == n_stages - 1:
            st = LLamaLastStage.__new__(LLamaLastStage)
            nn.Module.__init__(st)
            st.norm, st.head, st.vocab_size = model.last.norm, model.last.head, model.last.vocab_size
        else:
            st = LLamaStage.__new__(LLamaStage)
            nn.Module.__init__(st)
        st.layers = nn.ModuleList(mine)
        st.precision, st.act_dtype = model.precision, _act_dtype(model.precision)
        if n_stages == 1:
            st = model
        out.append(st)
    return out


def causalLLMLoss(logits, target, vocab_size=None, ignore_index=-100, scale: float = 1.0):  # noqa: N802
    """Next-token CE (reference name): logits[:, :-1] vs target[:, 1:]. On the device every row of
    the [B, S, V] logits goes to the fused kernel with the last position's label set to
    ``ignore_index`` (same mean, no copy of the [B, S-1, V] slice). ``scale`` (extension): a
    constant factor such as 1 / micro-batches, folded into the kernel's normaliser."""
    if not logits.is_cuda:
        return A.cross_entropy_vocab(logits[:, :-1].contiguous(), target[:, 1:].contiguous(), ignore_index,
                                     scale)
    lab = torch.empty(target.shape, dtype=torch.int32, device=target.device)
    lab[:, :-1] = target[:, 1:]
    lab[:, -1] = ignore_index
    return A.cross_entropy_vocab(logits, lab, ignore_index, scale)
