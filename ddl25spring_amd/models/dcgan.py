"""DCGAN generator / discriminator (Radford et al. 2015) for the federated-GAN config [NS].

The reference has no GAN (SURVEY M9 / BASELINE config "federated DCGAN"); this follows the
standard DCGAN recipe at CIFAR-10 shape (32x32x3): transposed-conv generator with BN+ReLU and a
tanh head, strided-conv discriminator with BN+LeakyReLU(0.2), N(0, 0.02) init, Adam(2e-4, 0.5).

MI355X mapping: activations NHWC; every conv / transposed conv is the implicit-GEMM MFMA kernel (a
stride-2 transposed conv IS the phase-decomposed dgrad kernel), BN statistics come from the conv
epilogue (discriminator) or one streaming pass (generator), BN+activation is one fused pass,
BCE-with-logits is one kernel. RGB is carried as 32 channels whose extra weights are zero (they
provably stay zero: their gradients are exactly zero), the 100-d latent as 128.

Precision (``precision=``): "fp32" (default: the reference's generative lab trains in fp32,
lab/tutorial_2a/generative-modeling.py:13-130) runs fp32 activations, weights and gradients on
the fp32 kernels (conv_f32.hip X6 / exact-fp32 MFMA, bn_f32.hip, a deterministic fp32 BCE);
"bf16" runs bf16 MFMA operands and activations with fp32 master weights.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from ..ops import autograd_ops as A


def _pad32(c: int) -> int:
    return (c + 31) // 32 * 32


PRECISIONS = ("fp32", "bf16")


def _act_dtype(precision: str):
    if precision not in PRECISIONS:
        raise ValueError(f"DCGAN precision must be one of {PRECISIONS}, got {precision!r}")
    return torch.float32 if precision == "fp32" else torch.bfloat16


class _BN(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.weight = nn.Parameter(torch.empty(c).normal_(1.0, 0.02))
        self.bias = nn.Parameter(torch.zeros(c))
        self.register_buffer("running_mean", torch.zeros(c))
        self.register_buffer("running_var", torch.ones(c))

    def forward(self, x, act, stats=None):
        return A.batch_norm_act(x, self.weight, self.bias, self.running_mean, self.running_var,
                                self.training, act=act, stats=stats)


class Generator(nn.Module):
    """z [N, nz] -> image NHWC [N, 32, 32, nc_pad] in [-1, 1] (channels >= nc are zero)."""

    def __init__(self, nz: int = 100, ngf: int = 64, nc: int = 3, precision: str = "fp32"):
        super().__init__()
        self.nz, self.nz_pad, self.nc, self.nc_pad, self.ngf = nz, _pad32(nz), nc, _pad32(nc), ngf
        self.precision, self.act_dtype = precision, _act_dtype(precision)
        c0 = 4 * ngf
        # ConvTranspose2d(nz, 4ngf, 4, 1, 0) on a 1x1 input == a linear to [4, 4, 4ngf] (NHWC)
        w0 = torch.zeros(16 * c0, self.nz_pad)
        w0[:, :nz].normal_(0.0, 0.02)
        self.proj = nn.Parameter(w0)
        self.bn0 = _BN(c0)
        self.up1 = nn.Parameter(torch.empty(c0, 4, 4, 2 * ngf).normal_(0.0, 0.02))
        self.bn1 = _BN(2 * ngf)
        self.up2 = nn.Parameter(torch.empty(2 * ngf, 4, 4, ngf).normal_(0.0, 0.02))
        self.bn2 = _BN(ngf)
        w3 = torch.zeros(ngf, 4, 4, self.nc_pad)
        w3[..., :nc].normal_(0.0, 0.02)
        self.up3 = nn.Parameter(w3)

    def forward(self, z):
        N = z.shape[0]
        if z.shape[1] != self.nz_pad:
            z = torch.cat([z, z.new_zeros(N, self.nz_pad - z.shape[1])], 1)
        if z.is_cuda:
            z = z.to(self.act_dtype)  # the activation dtype selects the kernels' precision
        h = A.linear(z, self.proj).view(N, 4, 4, 4 * self.ngf)
        h = self.bn0(h, "relu")
        h = self.bn1(A.conv_transpose2d(h, self.up1, 2, 1), "relu")      # 8x8
        h = self.bn2(A.conv_transpose2d(h, self.up2, 2, 1), "relu")      # 16x16
        return A.activation(A.conv_transpose2d(h, self.up3, 2, 1), "tanh")  # 32x32

    def sample(self, n, device=None, generator=None):
        dev = device or self.proj.device
        return self.forward(torch.randn(n, self.nz, device=dev, generator=generator))


class Discriminator(nn.Module):
    """image NHWC [N, 32, 32, nc_pad] -> logits [N, 32] (column 0 is the real/fake logit)."""

    def __init__(self, ndf: int = 64, nc: int = 3, precision: str = "fp32"):
        super().__init__()
        self.nc, self.nc_pad, self.ndf = nc, _pad32(nc), ndf
        self.precision, self.act_dtype = precision, _act_dtype(precision)
        w0 = torch.zeros(ndf, 4, 4, self.nc_pad)
        w0[..., :nc].normal_(0.0, 0.02)
        self.c0 = nn.Parameter(w0)
        self.c1 = nn.Parameter(torch.empty(2 * ndf, 4, 4, ndf).normal_(0.0, 0.02))
        self.bn1 = _BN(2 * ndf)
        self.c2 = nn.Parameter(torch.empty(4 * ndf, 4, 4, 2 * ndf).normal_(0.0, 0.02))
        self.bn2 = _BN(4 * ndf)
        # Conv2d(4ndf, 1, 4, 1, 0) on 4x4 == linear 16*4ndf -> 1, padded to 32 output rows
        wh = torch.zeros(32, 16 * 4 * ndf)
        wh[0].normal_(0.0, 0.02)
        self.head = nn.Parameter(wh)

    def forward(self, x):
        N = x.shape[0]
        if x.is_cuda:
            x = x.to(self.act_dtype)
        h = A.activation(A.conv2d(x, self.c0, 2, 1), "leaky_relu")   # 16x16
        y, st = A.conv2d(h, self.c1, 2, 1, with_stats=True)            # 8x8
        h = self.bn1(y, "leaky_relu", st)
        y, st = A.conv2d(h, self.c2, 2, 1, with_stats=True)            # 4x4
        h = self.bn2(y, "leaky_relu", st)
        return A.linear(h.reshape(N, -1), self.head)


def to_nhwc_padded(img_nchw: torch.Tensor, nc_pad: int = 32) -> torch.Tensor:
    """[N, C, H, W] float in [-1, 1] -> [N, H, W, nc_pad] (zero channels appended)."""
    x = img_nchw.permute(0, 2, 3, 1)
    if x.shape[-1] < nc_pad:
        x = torch.cat([x, x.new_zeros(*x.shape[:-1], nc_pad - x.shape[-1])], -1)
    return x.contiguous()


class GANTrainer:
    """One (D, G) step pair with the standard non-saturating losses; fused FlatAdam on device."""

    def __init__(self, gen: Generator, disc: Discriminator, lr: float = 2e-4, betas=(0.5, 0.999)):
        from ..optim import FlatAdam
        self.G, self.D = gen, disc
        dev = gen.proj.device
        mk = FlatAdam if dev.type == "cuda" else (lambda p, **kw: torch.optim.Adam(p, **kw))
        self.optG = mk(gen.parameters(), lr=lr, betas=betas)
        self.optD = mk(disc.parameters(), lr=lr, betas=betas)

    def step(self, real_nhwc: torch.Tensor, z: torch.Tensor | None = None):
        N = real_nhwc.shape[0]
        if z is None:
            z = torch.randn(N, self.G.nz, device=real_nhwc.device)
        # discriminator: real -> 1, fake -> 0
        self.optD.zero_grad()
        fake = self.G(z)
        lossD = A.bce_with_logits(self.D(real_nhwc), 1.0) + A.bce_with_logits(self.D(fake.detach()), 0.0)
        lossD.backward()
        self.optD.step()
        # generator: fool D (non-saturating)
        self.optG.zero_grad()
        lossG = A.bce_with_logits(self.D(fake), 1.0)
        lossG.backward()
        self.optG.step()
        return lossD.detach(), lossG.detach()


# ------------------------------------------------------------------------- client-batched
def _slots(t: torch.Tensor, S: int) -> torch.Tensor:
    return t.detach().unsqueeze(0).repeat(S, *([1] * t.dim())).clone()


class _GBN(nn.Module):
    def __init__(self, bn: _BN, S: int):
        super().__init__()
        self.weight = nn.Parameter(_slots(bn.weight, S))
        self.bias = nn.Parameter(_slots(bn.bias, S))
        self.register_buffer("running_mean", _slots(bn.running_mean, S))
        self.register_buffer("running_var", _slots(bn.running_var, S))

    def forward(self, x, act, stats=None):
        from ..ops import grouped as Gp
        return Gp.batch_norm_act(x, self.weight, self.bias, self.running_mean, self.running_var, self.training,
                                 act=act, stats=stats)


class GroupedGenerator(nn.Module):
    """S client copies of a Generator as slot tensors [S, ...]: z [G, N, nz] -> [G, N, 32, 32, nc_pad]
    for the first G slots, every layer one client-batched launch (ops/grouped.py). Parameter and
    buffer order match ``Generator``, so a slot row has a single generator's flat layout."""

    def __init__(self, gen: Generator, S: int):
        super().__init__()
        self.nz, self.nz_pad, self.nc, self.nc_pad, self.ngf = gen.nz, gen.nz_pad, gen.nc, gen.nc_pad, gen.ngf
        self.precision, self.act_dtype = gen.precision, gen.act_dtype
        self.proj = nn.Parameter(_slots(gen.proj, S))
        self.bn0 = _GBN(gen.bn0, S)
        self.up1 = nn.Parameter(_slots(gen.up1, S))
        self.bn1 = _GBN(gen.bn1, S)
        self.up2 = nn.Parameter(_slots(gen.up2, S))
        self.bn2 = _GBN(gen.bn2, S)
        self.up3 = nn.Parameter(_slots(gen.up3, S))

    def forward(self, z):
        from ..ops import grouped as Gp
        G, N = z.shape[:2]
        if z.shape[2] != self.nz_pad:
            z = torch.cat([z, z.new_zeros(G, N, self.nz_pad - z.shape[2])], 2)
        if z.is_cuda:
            z = z.to(self.act_dtype)
        h = Gp.linear(z, self.proj).view(G, N, 4, 4, 4 * self.ngf)
        h = self.bn0(h, "relu")
        h = self.bn1(Gp.conv_transpose2d(h, self.up1, 2, 1), "relu")
        h = self.bn2(Gp.conv_transpose2d(h, self.up2, 2, 1), "relu")
        return A.activation(Gp.conv_transpose2d(h, self.up3, 2, 1), "tanh")


class GroupedDiscriminator(nn.Module):
    """S client copies of a Discriminator: [G, N, 32, 32, nc_pad] -> logits [G, N, 32]."""

    def __init__(self, disc: Discriminator, S: int):
        super().__init__()
        self.nc, self.nc_pad, self.ndf = disc.nc, disc.nc_pad, disc.ndf
        self.precision, self.act_dtype = disc.precision, disc.act_dtype
        self.c0 = nn.Parameter(_slots(disc.c0, S))
        self.c1 = nn.Parameter(_slots(disc.c1, S))
        self.bn1 = _GBN(disc.bn1, S)
        self.c2 = nn.Parameter(_slots(disc.c2, S))
        self.bn2 = _GBN(disc.bn2, S)
        self.head = nn.Parameter(_slots(disc.head, S))

    def forward(self, x):
        from ..ops import grouped as Gp
        G, N = x.shape[:2]
        if x.is_cuda:
            x = x.to(self.act_dtype)
        h = A.activation(Gp.conv2d(x, self.c0, 2, 1), "leaky_relu")
        y, st = Gp.conv2d(h, self.c1, 2, 1, with_stats=True)
        h = self.bn1(y, "leaky_relu", st)
        y, st = Gp.conv2d(h, self.c2, 2, 1, with_stats=True)
        h = self.bn2(y, "leaky_relu", st)
        return Gp.linear(h.reshape(G, N, -1), self.head)


class GroupedGANTrainer:
    """One (D, G) step pair for the first G client slots at once: per-client non-saturating losses
    (the grouped BCE sums each client's own mean), SlotAdam per network (one launch each, per-client
    step counters)."""

    def __init__(self, gen: GroupedGenerator, disc: GroupedDiscriminator, S: int, lr: float = 2e-4,
                 betas=(0.5, 0.999)):
        from ..optim import SlotAdam
        self.G, self.D = gen, disc
        shadow = gen.proj.is_cuda and gen.precision == "bf16"  # fp32 kernels read the fp32 rows
        self.optG = SlotAdam(gen.parameters(), S, lr=lr, betas=betas, bf16_shadow=shadow)
        self.optD = SlotAdam(disc.parameters(), S, lr=lr, betas=betas, bf16_shadow=shadow)

    def step(self, real, z):
        """real [G, N, 32, 32, nc_pad], z [G, N, nz] -> (sum of the clients' D losses, of G losses)."""
        from ..ops import grouped as Gp
        G = real.shape[0]
        self.optD.zero_grad()
        fake = self.G(z)
        lossD = Gp.bce_with_logits(self.D(real), 1.0) + Gp.bce_with_logits(self.D(fake.detach()), 0.0)
        lossD.backward()
        self.optD.step(G)
        self.optG.zero_grad()
        lossG = Gp.bce_with_logits(self.D(fake), 1.0)
        lossG.backward()
        self.optG.step(G)
        return lossD.detach(), lossG.detach()
