"""Tabular models of the generative-modelling and vertical-FL labs (fp32, exact reference numerics).

These nets are a few thousand parameters on <= 1,025 rows, trained in exact fp32 like the
reference. On the device every layer is a fused HIP kernel of csrc/kernels/tabular.hip (linear +
bias + activation on fp32 MFMA, BatchNorm1d + activation, soft-target CE, MSE+KL, Philox
reparameterisation — ``ops/tabular_ops.py``); on the CPU the same modules run the identical torch
composition. Their optimizers can be the fused flat ``optim.FlatAdam`` and, in the vertical-FL
runtime, their cut-layer tensors cross GPUs over RCCL (``ddl25spring_amd.vfl``).

* ``HeartDiseaseNN``      — lab/tutorial_2a/centralized.py:13-28
* ``Autoencoder``+``customLoss`` — lab/tutorial_2a/generative-modeling.py:13-130 (tabular VAE;
  ``sample`` draws from the batch-averaged posterior N(mean mu, mean sigma))
* ``BottomModel`` / ``TopModel`` / ``VFLNetwork`` — lab/tutorial_2b/vfl.py:11-102
* ``ClientEncoder`` / ``ClientDecoder`` / ``ServerVAE`` / ``VFLVAE`` / ``combined_loss`` —
  lab/tutorial_2b/exercise_3.py:10-147
"""
from __future__ import annotations


import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import tabular_ops as TO
from ..optim import make_adam


class FLinear(nn.Linear):
    """nn.Linear with a fused activation ('none' | 'relu' | 'leaky_relu'); one kernel on device."""

    def __init__(self, in_features, out_features, act="none", slope=0.01, bias=True):
        super().__init__(in_features, out_features, bias=bias)
        self.act_kind, self.slope = act, slope

    def forward(self, x):
        return TO.linear_act(x, self.weight, self.bias, self.act_kind, self.slope)


class FBatchNorm1d(nn.BatchNorm1d):
    """nn.BatchNorm1d (batch statistics in training, running statistics in eval) + fused act."""

    def __init__(self, num_features, act="none", slope=0.01):
        super().__init__(num_features)
        self.act_kind, self.slope = act, slope

    def forward(self, x):
        if self.training:
            self.num_batches_tracked.add_(1)
        return TO.batch_norm1d_act(x, self.weight, self.bias, self.running_mean, self.running_var,
                                   self.training, self.momentum, self.eps, self.act_kind, self.slope)


class SoftCrossEntropy(nn.Module):
    """nn.CrossEntropyLoss (mean; hard labels or probability targets), fused on device."""

    def forward(self, logits, target):
        return TO.cross_entropy(logits, target)


def _mlp_bn(dims, final_act=True):
    layers = []
    for i, (a, b) in enumerate(zip(dims[:-1], dims[1:])):
        act = "relu" if (final_act or i < len(dims) - 2) else "none"
        layers += [FLinear(a, b), FBatchNorm1d(b, act)]
    return nn.Sequential(*layers)


class HeartDiseaseNN(nn.Module):
    def __init__(self, in_features: int = 30):
        super().__init__()
        self.fc1 = FLinear(in_features, 64, "leaky_relu")
        self.fc2 = FLinear(64, 128, "leaky_relu")
        self.fc3 = FLinear(128, 256, "leaky_relu")
        self.fc4 = FLinear(256, 2)
        self.dropout = nn.Dropout(0.1)

    def forward(self, x):
        return self.fc4(self.dropout(self.fc3(self.fc2(self.fc1(x)))))


def train_centralized(net, Xtr, ytr, Xte, yte, epochs: int = 49, optimizer=None):
    """Full-batch training keeping a DEEP copy of the best-test-accuracy weights (fixes the
    reference's aliasing ``best_params = net.state_dict()``, centralized.py:51,69-70 / SURVEY Q9).

    Sync-free: the best-epoch selection is a device-side ``torch.where`` over the state tensors
    (no per-epoch ``.item()``); the history is read back once at the end."""
    opt = optimizer or make_adam(net.parameters(), decoupled=True)
    crit = SoftCrossEntropy()
    dev = Xtr.device
    best = torch.full((), -1.0, device=dev)
    best_sd = {k: v.detach().clone() for k, v in net.state_dict().items()}
    losses, accs = [], []
    for _ in range(1, epochs + 1):
        net.train()
        opt.zero_grad()
        out = net(Xtr)
        loss = crit(out, ytr)
        loss.backward()
        opt.step()
        net.eval()  # the reference scores with dropout still active; we score the deterministic net
        with torch.no_grad():
            acc = (net(Xte).argmax(1) == yte).float().mean()
            better = acc > best
            for k, v in net.state_dict().items():
                best_sd[k].copy_(torch.where(better, v, best_sd[k]))
            best = torch.maximum(best, acc)
        losses.append(loss.detach())
        accs.append(acc)
    net.load_state_dict(best_sd)
    hist = list(zip(torch.stack(losses).tolist(), torch.stack(accs).tolist()))
    return float(best), hist


class Autoencoder(nn.Module):
    """Tabular VAE: encoder D->H->H2->H2->latent (BN+ReLU), mu/logvar heads, mirrored decoder."""

    def __init__(self, D_in, H=50, H2=12, latent_dim=3):
        super().__init__()
        self.enc = _mlp_bn([D_in, H, H2, H2, latent_dim])
        self.fc21, self.fc22 = FLinear(latent_dim, latent_dim), FLinear(latent_dim, latent_dim)
        self.dec = nn.Sequential(_mlp_bn([latent_dim, latent_dim, H2, H2, H]),
                                 FLinear(H, D_in), FBatchNorm1d(D_in))
        self.optimizer = self.criterion = None

    def encode(self, x):
        h = self.enc(x)
        return self.fc21(h), self.fc22(h)

    def reparameterize(self, mu, logvar):
        if self.training:
            return TO.reparameterize(mu, logvar)
        return mu

    def decode(self, z):
        return self.dec(z)

    def forward(self, x):
        mu, logvar = self.encode(x)
        return self.decode(self.reparameterize(mu, logvar)), mu, logvar

    def train_with_settings(self, epochs, batch_sz, real_data, optimizer, loss_fn,
                            zero_grad_per_batch: bool = True, log=None):
        """Mini-batch training. ``zero_grad_per_batch=False`` reproduces the reference's
        once-per-epoch zero_grad (gradient accumulation across the epoch)."""
        self.optimizer, self.criterion = optimizer, loss_fn
        n = len(real_data)
        nb = (n + batch_sz - 1) // batch_sz
        losses = []
        for epoch in range(epochs):
            self.train()
            if not zero_grad_per_batch:
                optimizer.zero_grad()
            total = torch.zeros((), device=real_data.device)
            for b in range(nb):
                mb = real_data[b * batch_sz:(b + 1) * batch_sz]
                if zero_grad_per_batch:
                    optimizer.zero_grad()
                out, mu, logvar = self(mb)
                loss = loss_fn(out, mb, mu, logvar)
                loss.backward()
                optimizer.step()
                total += loss.detach()  # accumulated on the device: no per-batch host sync
            losses.append(total / nb)
            if log:
                log(epoch, float(losses[-1]))
        return torch.stack(losses).tolist()

    @torch.no_grad()
    def sample(self, nr_samples, dims, logvar, mu, label_col: bool = True, eval_mode: bool = False):
        """Decode draws from N(mean(mu), mean(sigma)) (the batch-averaged posterior, as the
        reference does); clip+round the label column. The reference decodes in whatever mode the
        model is in (train -> BN uses the sample batch's statistics); ``eval_mode`` switches to
        running statistics."""
        sigma = torch.exp(logvar / 2)
        q = torch.distributions.Normal(mu.mean(0), sigma.mean(0))
        z = q.rsample((nr_samples,))
        if eval_mode:
            self.eval()
        pred = self.decode(z).cpu().numpy()
        if label_col:
            pred[:, -1] = np.round(np.clip(pred[:, -1], 0, 1))
        return pred


class customLoss(nn.Module):  # noqa: N801 - reference name
    """MSE(sum) + KL — one fused reduction with its gradients on the device."""

    def forward(self, x_recon, x, mu, logvar):
        return TO.mse_kl(x_recon, x, mu, logvar)


# ----------------------------------------------------------------------------------- split-NN
class BottomModel(nn.Module):
    def __init__(self, in_feat, out_feat):
        super().__init__()
        self.local_out_dim = out_feat
        self.fc1 = FLinear(in_feat, out_feat, "relu")
        self.fc2 = FLinear(out_feat, out_feat, "relu")
        self.dropout = nn.Dropout(0.1)

    def forward(self, x):
        return self.dropout(self.fc2(self.fc1(x)))


class TopModel(nn.Module):
    """concat -> 128 -> 256 -> 2, LeakyReLU after EVERY layer incl. the logits, then Dropout
    (kept: it is the reference architecture, vfl.py:35-40 / SURVEY Q7)."""

    def __init__(self, local_models, n_outs=2):
        super().__init__()
        self.in_size = sum(m.local_out_dim for m in local_models)
        self.fc1 = FLinear(self.in_size, 128, "leaky_relu")
        self.fc2 = FLinear(128, 256, "leaky_relu")
        self.fc3 = FLinear(256, n_outs, "leaky_relu")
        self.dropout = nn.Dropout(0.1)

    def forward(self, xs):
        x = torch.cat(xs, 1) if isinstance(xs, (list, tuple)) else xs
        return self.dropout(self.fc3(self.fc2(self.fc1(x))))


class VFLNetwork(nn.Module):
    """Single-process split-NN. Defaults fix the reference's quirks; each can be restored on its
    own, or all at once with ``parity=True``: ``register_bottoms=False`` keeps the bottom models in
    a plain list (never optimised, Q5), ``zero_grad_per_batch=False`` zeroes once per epoch
    (gradient accumulation, Q6), ``eval_in_test=False`` tests with dropout active (Q8)."""

    def __init__(self, local_models, n_outs=2, parity: bool = False, lr: float = 1e-3,
                 register_bottoms: bool | None = None, zero_grad_per_batch: bool | None = None,
                 eval_in_test: bool | None = None):
        super().__init__()
        pick = lambda v: (not parity) if v is None else v  # noqa: E731
        self.register_bottoms, self.zero_grad_per_batch = pick(register_bottoms), pick(zero_grad_per_batch)
        self.eval_in_test = pick(eval_in_test)
        if not self.register_bottoms:
            self.bottom_models = list(local_models)
        else:
            self.bottom_models = nn.ModuleList(local_models)
        self.top_model = TopModel(local_models, n_outs)
        self.lr, self._opt = lr, None
        self.criterion = SoftCrossEntropy()
        self.num_cli = self.cli_features = None

    @property
    def optimizer(self):
        """AdamW over the registered parameters (vfl.py:50), built on first use so it sees the
        device the network was moved to: the fused FlatAdam on the GPU."""
        if self._opt is None:
            self._opt = make_adam(self.parameters(), lr=self.lr, decoupled=True)
        return self._opt

    @optimizer.setter
    def optimizer(self, opt):
        self._opt = opt

    def forward(self, xs):
        return self.top_model([m(x) for m, x in zip(self.bottom_models, xs)])

    def _tensors(self, x, y, cli_features):
        xs = [torch.tensor(x[f].values.astype(np.float32)) for f in cli_features]
        yt = torch.tensor(y.values.astype(np.float32))
        dev = next(self.parameters()).device
        return [t.to(dev).contiguous() for t in xs], yt.to(dev).contiguous()

    def fused_epoch_engine(self, batch_sz):
        """The one-launch epoch engine (ops/mlp_epoch.py, csrc/kernels/mlp_epoch.hip) when this net
        and its optimizer fit it: on the GPU, FlatAdamW over exactly the bottoms + top, gradients
        zeroed per mini-batch, bottoms registered; else None (the module path runs)."""
        from ..ops import mlp_epoch as ME
        from ..optim import FlatAdam
        opt = self.optimizer
        if not (ME.ENABLED[0] and self.zero_grad_per_batch and self.register_bottoms
                and isinstance(opt, FlatAdam) and opt.data.is_cuda):
            return None
        key = (batch_sz, id(opt))
        eng = getattr(self, "_fused", None)
        if eng is None or eng[0] != key:
            try:
                eng = (key, ME.MlpEpoch(ME.splitnn_graph(list(self.bottom_models), self.top_model), opt, batch_sz))
            except (TypeError, ValueError):
                eng = (key, None)
            self._fused = eng
        return eng[1]

    def train_with_settings(self, epochs, batch_sz, n_cli, cli_features, x, y, log_loss=None,
                            verbose=False):
        self.num_cli, self.cli_features = n_cli, cli_features
        xs, yt = self._tensors(x, y, cli_features)
        n = len(yt)
        nb = (n + batch_sz - 1) // batch_sz
        hist = []
        eng = self.fused_epoch_engine(batch_sz)
        for epoch in range(epochs):
            if eng is not None:  # the whole epoch in one launch; loss / correct stay on the device
                stats = torch.zeros(2, device=yt.device)
                eng.run(xs, yt, stats)
                hist.append(stats / torch.tensor([float(nb), float(n)], device=yt.device))
                if log_loss is not None:
                    log_loss(float(hist[-1][0]))
                if verbose:
                    l, a = hist[-1].tolist()
                    print(f"Epoch: {epoch} Train accuracy: {100 * a:.2f}% Loss: {l:.3f}")
                continue
            self.train()
            for m in self.bottom_models:
                m.train()
            if not self.zero_grad_per_batch:
                self.optimizer.zero_grad()
            # loss / correct accumulate on the device; the host reads them once (at the end, or
            # per epoch only when a logger asks)
            total = torch.zeros((), device=yt.device)
            correct = torch.zeros((), dtype=torch.int64, device=yt.device)
            for b in range(nb):
                sl = slice(b * batch_sz, (b + 1) * batch_sz)
                if self.zero_grad_per_batch:
                    self.optimizer.zero_grad()
                outs = self.forward([t[sl] for t in xs])
                loss = self.criterion(outs, yt[sl])
                loss.backward()
                self.optimizer.step()
                total += loss.detach()
                correct += (outs.argmax(1) == yt[sl].argmax(1)).sum()
            hist.append(torch.stack([total / nb, correct / n]))
            if log_loss is not None:
                log_loss(float(hist[-1][0]))
            if verbose:
                l, a = hist[-1].tolist()
                print(f"Epoch: {epoch} Train accuracy: {100 * a:.2f}% Loss: {l:.3f}")
        return [tuple(h) for h in torch.stack(hist).tolist()]

    def test(self, x, y):
        xs, yt = self._tensors(x, y, self.cli_features)
        if self.eval_in_test:
            self.eval()
            for m in self.bottom_models:
                m.eval()
        with torch.no_grad():
            outs = self.forward(xs)
            acc = (outs.argmax(1) == yt.argmax(1)).float().mean()
            loss = self.criterion(outs, yt)
        return acc, loss


# ------------------------------------------------------------------------------------ VFL-VAE
class ClientEncoder(nn.Module):
    def __init__(self, input_dim, latent_dim):
        super().__init__()
        self.net = _mlp_bn([input_dim, 48, 32, 32, latent_dim], final_act=True)

    def forward(self, x):
        return self.net(x)


class ClientDecoder(nn.Module):
    def __init__(self, latent_dim, output_dim):
        super().__init__()
        self.net = nn.Sequential(_mlp_bn([latent_dim, latent_dim, 32, 48]),
                                 FLinear(48, output_dim), FBatchNorm1d(output_dim))

    def forward(self, z):
        return self.net(z)


class ServerVAE(nn.Module):
    def __init__(self, D_in, H=48, H2=32, latent_dim=16):
        super().__init__()
        self.enc = _mlp_bn([D_in, H, H2, H2, latent_dim])
        self.fc21, self.fc22 = FLinear(latent_dim, latent_dim), FLinear(latent_dim, latent_dim)
        self.dec = nn.Sequential(_mlp_bn([latent_dim, latent_dim, H2, H2, H]),
                                 FLinear(H, D_in), FBatchNorm1d(D_in))

    def encode(self, x):
        h = self.enc(x)
        return self.fc21(h), self.fc22(h)

    def reparameterize(self, mu, logvar):
        if self.training:
            return TO.reparameterize(mu, logvar)
        return mu

    def decode(self, z):
        return self.dec(z)

    def forward(self, x):
        mu, logvar = self.encode(x)
        return self.decode(self.reparameterize(mu, logvar)), mu, logvar


class VFLVAE(nn.Module):
    def __init__(self, client_encoders, server_vae, client_decoders, client_latent_dim):
        super().__init__()
        self.client_encoders = nn.ModuleList(client_encoders)
        self.server_vae = server_vae
        self.client_decoders = nn.ModuleList(client_decoders)
        self.client_latent_dim = client_latent_dim

    def forward(self, x_clients):
        lat = torch.cat([e(x) for e, x in zip(self.client_encoders, x_clients)], 1)
        recon_concat, mu, logvar = self.server_vae(lat)
        d = self.client_latent_dim
        recon = [dec(recon_concat[:, i * d:(i + 1) * d]) for i, dec in enumerate(self.client_decoders)]
        return recon, mu, logvar, lat, recon_concat


def combined_loss(x_clients, recon_clients, concat_latent, recon_concat, mu, logvar):
    client = sum(F.mse_loss(r, x, reduction="sum") for x, r in zip(x_clients, recon_clients))
    return client + TO.mse_kl(recon_concat, concat_latent, mu, logvar)
