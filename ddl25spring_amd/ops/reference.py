"""Pure-PyTorch reference implementations of every native op (fp32 math on bf16 storage).

Used (a) as the CPU execution path so the whole framework runs in GPU-less CI, and (b) as the
numerics oracle for the HIP kernels in ``tests/test_kernels_gpu.py``. They follow the same
layout contract as the kernels: NHWC activations with a leading client-group dimension
``[G, N, H, W, C]``, bf16 storage, fp32 accumulation.
"""
from __future__ import annotations

import contextlib

import numpy as np
import torch
import torch.nn.functional as F

# activation storage dtype of the CPU path: bf16 (mirrors the device numerics) or fp32 (a net in
# the fp32 precision mode runs its CPU ops inside ``storage(torch.float32)``)
_STORAGE = [torch.bfloat16]


def _bf(t: torch.Tensor) -> torch.Tensor:
    return t.to(_STORAGE[-1])


@contextlib.contextmanager
def storage(dtype):
    _STORAGE.append(dtype)
    try:
        yield
    finally:
        _STORAGE.pop()


def nhwc_to_nchw(x: torch.Tensor) -> torch.Tensor:
    return x.permute(0, 3, 1, 2)


def nchw_to_nhwc(x: torch.Tensor) -> torch.Tensor:
    return x.permute(0, 2, 3, 1)


def _is_gemm(geom) -> bool:
    """1x1 / stride 1 / no padding (every Linear layer): the conv is a plain GEMM over pixels."""
    return geom.R == 1 and geom.S == 1 and geom.stride == 1 and geom.pad == 0


def conv_fwd(x, w, geom, bias=None, relu=False, stats=None):
    G = geom.G
    if _is_gemm(geom):  # one batched matmul over the client groups (the CPU MLP path)
        y = torch.bmm(x.float().reshape(G, -1, geom.C), w.float().reshape(G, geom.K, geom.C).transpose(1, 2))
        if bias is not None:
            y = y + bias.float().reshape(G, 1, geom.K)
        if relu:
            y = y.clamp_min(0)
        if stats is not None:
            st = stats[:, 0] if stats.dim() == 4 else stats
            st[:, 0] += y.sum(1)
            st[:, 1] += (y * y).sum(1)
        return _bf(y).reshape(G, geom.N, geom.P, geom.Q, geom.K)
    outs = []
    for g in range(G):
        xi = nhwc_to_nchw(x[g].float())
        wi = w[g].float().permute(0, 3, 1, 2)  # [K, C, R, S]
        y = F.conv2d(xi, wi, None, geom.stride, geom.pad)
        y = nchw_to_nhwc(y)
        if bias is not None:
            y = y + bias[g].float()
        if relu:
            y = y.clamp_min(0)
        if stats is not None:
            flat = y.reshape(-1, geom.K)
            st = stats[g, 0] if stats.dim() == 4 else stats[g]
            st[0] += flat.sum(0)
            st[1] += (flat * flat).sum(0)
        outs.append(y)
    return _bf(torch.stack(outs)).contiguous()


def conv_dgrad(dy, w, geom, residual=None, mask=None):
    if _is_gemm(geom):
        G = geom.G
        dx = torch.bmm(dy.float().reshape(G, -1, geom.K), w.float().reshape(G, geom.K, geom.C))
        dx = dx.reshape(G, geom.N, geom.H, geom.W, geom.C)
        if residual is not None:
            dx = dx + residual.float()
        if mask is not None:
            dx = dx * (mask.float() > 0)
        return _bf(dx).contiguous()
    outs = []
    for g in range(geom.G):
        dyi = nhwc_to_nchw(dy[g].float())
        wi = w[g].float().permute(0, 3, 1, 2)
        dx = torch.nn.grad.conv2d_input((geom.N, geom.C, geom.H, geom.W), wi, dyi, geom.stride,
                                        geom.pad)
        dx = nchw_to_nhwc(dx)
        if residual is not None:
            dx = dx + residual[g].float()
        if mask is not None:
            dx = dx * (mask[g].float() > 0)
        outs.append(dx)
    return _bf(torch.stack(outs)).contiguous()


def conv_wgrad(dy, x, geom, dw, accumulate=True, scale=1.0):
    if _is_gemm(geom):
        G = geom.G
        gw = torch.bmm(dy.float().reshape(G, -1, geom.K).transpose(1, 2), x.float().reshape(G, -1, geom.C))
        gw = gw.reshape(G, geom.K, 1, 1, geom.C)
        if scale != 1.0:
            gw = gw * scale
        if accumulate:
            dw += gw
        else:
            dw.copy_(gw)
        return
    for g in range(geom.G):
        dyi = nhwc_to_nchw(dy[g].float())
        xi = nhwc_to_nchw(x[g].float())
        gw = torch.nn.grad.conv2d_weight(xi, (geom.K, geom.C, geom.R, geom.S), dyi, geom.stride,
                                         geom.pad)
        gw = gw.permute(0, 2, 3, 1)  # [K, R, S, C]
        if scale != 1.0:
            gw = gw * scale
        if accumulate:
            dw[g] += gw
        else:
            dw[g].copy_(gw)


def bn_finalize(stats, gamma, beta, running_mean, running_var, count, eps, momentum, training):
    if stats.dim() == 4:  # striped [G, S, 2, C]
        stats = stats.sum(1)
    if training:
        mean = stats[:, 0] / count
        var = (stats[:, 1] / count - mean * mean).clamp_min(0)
        if running_mean is not None:
            unb = var * count / max(count - 1, 1)
            running_mean.mul_(1 - momentum).add_(momentum * mean)
            running_var.mul_(1 - momentum).add_(momentum * unb)
    else:
        mean = running_mean.clone()
        var = running_var.clone()
    rstd = torch.rsqrt(var + eps)
    ga = gamma if gamma is not None else torch.ones_like(mean)
    be = beta if beta is not None else torch.zeros_like(mean)
    scale = ga * rstd
    shift = be - mean * scale
    return scale.contiguous(), shift.contiguous(), mean.contiguous(), rstd.contiguous()


def _act(y, act, slope=0.01):
    if act == 1:
        return y.clamp_min(0)
    if act == 2:
        return torch.where(y > 0, y, slope * y)
    if act == 3:
        return torch.tanh(y)
    if act == 4:
        return torch.sigmoid(y)
    return y


def _bn_act(y, act):
    # bn_apply's act code 3 is leaky(0.2) (act_fwd's 3 is tanh)
    return torch.where(y > 0, y, 0.2 * y) if act == 3 else _act(y, act)


def _bcast(v, x):
    # v [G, C] -> broadcast over x [G, ..., C]
    shape = [v.shape[0]] + [1] * (x.dim() - 2) + [v.shape[1]]
    return v.reshape(shape)


def bn_apply(x, scale, shift, r=None, rscale=None, rshift=None, act=0):
    y = x.float() * _bcast(scale, x) + _bcast(shift, x)
    if r is not None:
        rv = r.float()
        if rscale is not None:
            rv = rv * _bcast(rscale, x) + _bcast(rshift, x)
        y = y + rv
    return _bf(_bn_act(y, act)).contiguous()


def bn_bwd_reduce(dy, ymask, x, mean, rstd, dgamma=None, dbeta=None):
    d = dy.float()
    if ymask is not None:
        d = d * (ymask.float() > 0)
    xh = (x.float() - _bcast(mean, x)) * _bcast(rstd, x)
    dims = tuple(range(1, x.dim() - 1))
    s0 = d.sum(dims)
    s1 = (d * xh).sum(dims)
    if dbeta is not None:
        dbeta += s0
    if dgamma is not None:
        dgamma += s1
    return torch.stack([s0, s1], 1)


def bn_bwd_apply(dy, ymask, x, mean, rstd, gamma, sums, emit_dym=False):
    d = dy.float()
    if ymask is not None:
        d = d * (ymask.float() > 0)
    M = x[0].numel() // x.shape[-1]
    xh = (x.float() - _bcast(mean, x)) * _bcast(rstd, x)
    ga = gamma if gamma is not None else torch.ones_like(mean)
    dx = _bcast(ga * rstd, x) * (d - _bcast(sums[:, 0], x) / M - xh * _bcast(sums[:, 1], x) / M)
    dxb = _bf(dx).contiguous()
    if emit_dym:
        return dxb, _bf(d).contiguous()
    return dxb


def maxpool2_fwd(x):
    G, N, H, W, C = x.shape
    xi = x.float().reshape(G * N, H, W, C).permute(0, 3, 1, 2)
    y = F.max_pool2d(xi, 2)
    return _bf(y.permute(0, 2, 3, 1).reshape(G, N, H // 2, W // 2, C)).contiguous()


def maxpool2_bwd(x, dy):
    G, N, H, W, C = x.shape
    with torch.enable_grad():  # may be called from inside an autograd backward
        xi = x.float().reshape(G * N, H, W, C).permute(0, 3, 1, 2).detach().requires_grad_(True)
        y = F.max_pool2d(xi, 2)
        g = dy.float().reshape(G * N, H // 2, W // 2, C).permute(0, 3, 1, 2)
        (dx,) = torch.autograd.grad(y, xi, g)
    return _bf(dx.permute(0, 2, 3, 1).reshape(G, N, H, W, C)).contiguous()


def avgpool_fwd(x):
    G, N, H, W, C = x.shape
    return _bf(x.float().mean((2, 3))).contiguous()


def avgpool_bwd(dy, H, W):
    G, N, C = dy.shape
    return _bf((dy.float() / (H * W)).reshape(G, N, 1, 1, C).expand(G, N, H, W, C)).contiguous()


def dropout_mask(shape, p, seed, offset, device):
    g = torch.Generator(device="cpu")
    g.manual_seed((int(seed) * 1000003 + int(offset)) % (2 ** 63))
    return (torch.rand(shape, generator=g) > p).to(device)


def dropout(x, p, seed, offset):
    if p <= 0:
        return x.clone()
    m = dropout_mask(x.shape, p, seed, offset, x.device)
    return _bf(x.float() * m / (1 - p)).contiguous()


def act_fwd(x, act, slope=0.01):
    return _bf(_act(x.float(), act, slope)).contiguous()


def act_bwd(y, dy, act, slope=0.01):
    yf = y.float()
    d = dy.float()
    if act == 1:
        d = d * (yf > 0)
    elif act == 3:
        d = d * (1 - yf * yf)
    elif act == 4:
        d = d * yf * (1 - yf)
    else:
        d = torch.where(yf > 0, d, slope * d)
    return _bf(d).contiguous()


def bn_stats(x, stats):
    C = x.shape[-1]
    xf = x.float().reshape(x.shape[0], -1, C)
    st = stats[:, 0] if stats.dim() == 4 else stats
    st[:, 0] += xf.sum(1)
    st[:, 1] += (xf * xf).sum(1)


def bce_logits(l, t):
    """-> (sum loss, dloss/dl)."""
    loss = (l.clamp_min(0) - l * t + torch.log1p(torch.exp(-l.abs()))).sum()
    return loss, torch.sigmoid(l) - t


def channel_sum(x, out):
    C = x.shape[-1]
    out += x.float().reshape(x.shape[0], -1, C).sum(1)


def ce_fwd_bwd(logits, labels, targets, ncls, scale, loss=None, correct=None, want_grad=True):
    # logits [G, N, ld]
    z = logits.float()[..., :ncls]
    lse = torch.logsumexp(z, -1, keepdim=True)
    logp = z - lse
    if targets is not None:
        t = targets.float()
        lrow = -(t * logp).sum(-1)
        tsum = t.sum(-1, keepdim=True)
        grad = torch.exp(logp) * tsum - t
        ytrue = t.argmax(-1)
    else:
        lrow = -logp.gather(-1, labels.long().unsqueeze(-1)).squeeze(-1)
        grad = torch.exp(logp)
        grad.scatter_add_(-1, labels.long().unsqueeze(-1), -torch.ones_like(lrow).unsqueeze(-1))
        ytrue = labels.long()
    if loss is not None:
        loss += lrow.sum(-1) * scale
    if correct is not None:
        correct += (z.argmax(-1) == ytrue).sum(-1).to(correct.dtype)
    if not want_grad:
        return None
    full = torch.zeros_like(logits, dtype=torch.float32)
    full[..., :ncls] = grad * scale
    return _bf(full).contiguous()


def sgd(p, g, mom, shadow, lr, wd, momentum, dampening, nesterov, first_step, grad_scale=1.0):
    d = g * grad_scale + wd * p
    if momentum != 0:
        if first_step:
            mom.copy_(d)
        else:
            mom.mul_(momentum).add_((1 - dampening) * d)
        d = d + momentum * mom if nesterov else mom
    p.sub_(lr * d)
    if shadow is not None:
        shadow.copy_(p.to(shadow.dtype))


def sgd_direct(p, g, shadow, dmap, lr, grad_scale=1.0):
    """Columns marked in ``dmap`` (per 16) were updated inside the backward: shadow refresh only;
    the rest take a plain SGD step and have their gradient zeroed (optim.hip sgd_direct_kernel)."""
    rest = (dmap == 0).repeat_interleave(16).to(p.device)
    p[:, rest] -= lr * grad_scale * g[:, rest]
    g[:, rest] = 0
    if shadow is not None:
        shadow.copy_(p.to(shadow.dtype))


def adam(p, g, m, v, shadow, lr, beta1, beta2, eps, wd, step, decoupled, grad_scale=1.0):
    g = g * grad_scale
    if decoupled:
        p.mul_(1 - lr * wd)
    else:
        g = g + wd * p
    m.mul_(beta1).add_((1 - beta1) * g)
    v.mul_(beta2).add_((1 - beta2) * g * g)
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    denom = v.sqrt() / (bc2 ** 0.5) + eps
    p.sub_((lr / bc1) * m / denom)
    if shadow is not None:
        shadow.copy_(p.to(shadow.dtype))


def weighted_sum(src, coeff, out, accumulate=False):
    r = (coeff.reshape(-1, 1).to(src.dtype) * src).sum(0)
    if accumulate:
        out += r
    else:
        out.copy_(r)


def broadcast_rows(src, dst, shadow=None):
    dst.copy_(src.unsqueeze(0).expand_as(dst))
    if shadow is not None:
        shadow.copy_(dst.to(shadow.dtype))


def gram(X, center=None):
    Xc = X - center if center is not None else X
    return Xc @ Xc.t()


def coord_select(X, mode, trim=0):
    s, _ = torch.sort(X, 0)
    K = X.shape[0]
    if mode == 0:
        return 0.5 * (s[(K - 1) // 2] + s[K // 2])
    return s[trim:K - trim].mean(0)


def mse_kl(xr, x, mu, lv, kl_w=1.0):
    mse = ((xr - x) ** 2).sum()
    kl = -0.5 * (1 + lv - mu * mu - lv.exp()).sum()
    return mse + kl_w * kl


# ------------------------------------------------------------------------- Philox (numpy twin)
_M0, _M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
_W0, _W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)


def philox4x32(c0, c1, c2, c3, k0, k1):
    """Philox-4x32-10 on uint32 arrays (csrc/include/ddl_common.h philox4x32)."""
    c0, c1, c2, c3 = (np.asarray(v, dtype=np.uint32) for v in (c0, c1, c2, c3))
    k0, k1 = np.uint32(k0), np.uint32(k1)
    for _ in range(10):
        p0 = _M0 * c0.astype(np.uint64)
        p1 = _M1 * c2.astype(np.uint64)
        hi0, lo0 = (p0 >> np.uint64(32)).astype(np.uint32), p0.astype(np.uint32)
        hi1, lo1 = (p1 >> np.uint64(32)).astype(np.uint32), p1.astype(np.uint32)
        c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
        k0 = np.uint32((int(k0) + int(_W0)) & 0xFFFFFFFF)
        k1 = np.uint32((int(k1) + int(_W1)) & 0xFFFFFFFF)
    return c0, c1, c2, c3


def _unit(x):  # (0, 1], u32_to_unit
    return ((x >> np.uint32(8)).astype(np.float32) + np.float32(1.0)) * np.float32(1.0 / 16777216.0)


def gan_inputs(desc, steps: int, B: int, nz: int):
    """nn_ops.hip gan_inputs_kernel on the host: desc [(seed, n, off), ...] per slot ->
    (idx int64 [steps, G*B], z fp32 [steps, G, B, nz])."""
    G = len(desc)
    idx = np.empty((steps, G * B), dtype=np.int64)
    z = np.empty((steps, G, B, nz), dtype=np.float32)
    for g, (seed, n, off) in enumerate(desc):
        k0, k1 = int(seed) & 0xFFFFFFFF, (int(seed) >> 32) & 0xFFFFFFFF
        e = np.arange(steps * B, dtype=np.uint64)
        zeros = np.zeros_like(e, dtype=np.uint32)
        r = philox4x32(e.astype(np.uint32), (e >> np.uint64(32)).astype(np.uint32), zeros + np.uint32(0x1d872b41),
                       zeros, k0, k1)
        u = (r[0].astype(np.uint64) * np.uint64(n)) >> np.uint64(32)
        idx[:, g * B:(g + 1) * B] = (u.astype(np.int64) + int(off)).reshape(steps, B)
        e = np.arange(steps * B * nz, dtype=np.uint64)
        zeros = np.zeros_like(e, dtype=np.uint32)
        r = philox4x32(e.astype(np.uint32), (e >> np.uint64(32)).astype(np.uint32), zeros + np.uint32(0x6a09e667),
                       zeros, k0, k1)
        u1 = np.maximum(_unit(r[0]), np.float32(1e-12))
        u2 = _unit(r[1])
        zz = np.sqrt(np.float32(-2.0) * np.log(u1)) * np.cos(np.float32(6.28318530717958648) * u2)
        z[:, g] = zz.astype(np.float32).reshape(steps, B, nz)
    return torch.from_numpy(idx), torch.from_numpy(z)
