"""Vertical FL / tabular generative programs (reference lab/tutorial_2a, lab/tutorial_2b).

  centralized  HeartDiseaseNN full-batch AdamW, best-epoch weights kept (centralized.py)
  splitnn      VFLNetwork over a feature partition (vfl.py, exercise_1/2.py); with world > 1 the
               parties run one per rank and rank 0 holds the top model (vfl.splitnn)
  vae          tabular VAE + synthetic-data utility check (generative-modeling.py)
  vflvae       VFL-VAE (exercise_3.py)
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch


@dataclass
class VFLConfig:
    task: str = "splitnn"
    parties: int = 4
    partition: str = "raw"      # raw (D4) | random (D5, seed 42+i) | balanced (D6)
    perm_seed: int = 42
    epochs: int = 300
    batch_size: int = 64
    parity: bool = False        # reproduce the reference's quirks (Q5/Q6/Q8)
    seed: int = 42
    latent: int = 8
    ckpt_dir: str = ""          # distributed split-NN: per-rank sharded checkpoint (resumes if committed)
    ckpt_every: int = 0         # commit every N epochs (0: only at the end)


def _partition(cfg, df, X):
    from ..data import heart as H
    cols = list(X.columns)
    if cfg.partition == "raw":
        return H.partition_raw_columns(list(df.columns), cols, cfg.parties)
    if cfg.partition == "random":
        return H.partition_random(cols, cfg.parties, cfg.perm_seed)
    return H.partition_balanced(cols, cfg.parties)


def run_vfl(cfg: VFLConfig, ctx, log=print) -> dict:
    from ..data import heart as H
    from ..models import tabular as T
    from ..optim import make_adam
    df, real = H.load_heart()
    torch.manual_seed(cfg.seed)
    np.random.seed(cfg.seed)
    dev = ctx.device
    out = {"real_data": real}
    if cfg.task == "centralized":
        Xtr, Xte, ytr, yte = (torch.tensor(a).to(dev) for a in H.centralized_split(df))
        net = T.HeartDiseaseNN().to(dev)
        best, hist = T.train_centralized(net, Xtr, ytr.long(), Xte, yte.long(), epochs=cfg.epochs)
        out.update(best_test_accuracy=best)
    elif cfg.task == "splitnn":
        X, Y = H.vfl_frame(df)
        parts = _partition(cfg, df, X)
        Xtr, Xte = H.row_split(X)
        Ytr, Yte = H.row_split(Y)
        if ctx.world > 1:
            out.update(_distributed_splitnn(cfg, ctx, parts, Xtr, Ytr, Xte, Yte))
        else:
            net = T.VFLNetwork([T.BottomModel(len(p), 2 * len(p)) for p in parts], 2,
                               parity=cfg.parity).to(dev)
            hist = net.train_with_settings(cfg.epochs, cfg.batch_size, cfg.parties, parts, Xtr, Ytr)
            acc, loss = net.test(Xte, Yte)
            out.update(train_loss=hist[-1][0], train_accuracy=hist[-1][1],
                       test_accuracy=float(acc), test_loss=float(loss))
    elif cfg.task == "vae":
        Xtr, Xte, ytr, yte = H.centralized_split(df, scaler="standard")
        real_t = torch.cat([torch.tensor(Xtr), torch.tensor(ytr).float().view(-1, 1)], 1).to(dev)
        vae = T.Autoencoder(real_t.shape[1], 48, 32, 16).to(dev)
        opt = make_adam(vae.parameters(), lr=1e-3)
        losses = vae.train_with_settings(cfg.epochs, cfg.batch_size, real_t, opt, T.customLoss(),
                                         zero_grad_per_batch=not cfg.parity)
        _, mu, logvar = vae(real_t)
        syn = vae.sample(len(real_t), mu.shape[1], logvar, mu)
        sx, sy = torch.tensor(syn[:, :-1]).to(dev), torch.tensor(syn[:, -1]).long().to(dev)
        Xte_t, yte_t = torch.tensor(Xte).to(dev), torch.tensor(yte).long().to(dev)
        r_best, _ = T.train_centralized(T.HeartDiseaseNN().to(dev), real_t[:, :-1],
                                        real_t[:, -1].long(), Xte_t, yte_t)
        s_best, _ = T.train_centralized(T.HeartDiseaseNN().to(dev), sx, sy, Xte_t, yte_t)
        out.update(final_loss=losses[-1], real_trained_acc=r_best, synthetic_trained_acc=s_best)
    elif cfg.task == "vflvae":
        std = H.standard_frame(df)
        parts = H.partition_balanced(list(std.columns), cfg.parties)
        xs = [torch.tensor(std[p].values).float().to(dev) for p in parts]
        m = T.VFLVAE([T.ClientEncoder(len(p), cfg.latent) for p in parts],
                     T.ServerVAE(cfg.parties * cfg.latent, 48, 32, 16),
                     [T.ClientDecoder(cfg.latent, len(p)) for p in parts], cfg.latent).to(dev)
        opt = make_adam(m.parameters(), lr=1e-3)
        losses = []
        for _ in range(cfg.epochs):
            opt.zero_grad()
            rc, mu, lv, lat, rcat = m(xs)
            loss = T.combined_loss(xs, rc, lat, rcat, mu, lv)
            loss.backward()
            opt.step()
            losses.append(loss.detach())
        losses = torch.stack(losses).tolist()  # one host read for the whole run
        out.update(first_loss=losses[0], final_loss=losses[-1])
    else:
        raise ValueError(cfg.task)
    if log and ctx.rank == 0:
        log({k: (round(v, 4) if isinstance(v, float) else v) for k, v in out.items()})
    return out


def _distributed_splitnn(cfg, ctx, parts, Xtr, Ytr, Xte, Yte):
    """Rank 0 = label holder / top model, ranks 1..P = parties (world = P + 1)."""
    from ..models import tabular as T
    from ..vfl.splitnn import SplitNNParty, SplitNNServer
    if ctx.world != cfg.parties + 1:
        raise ValueError(f"distributed split-NN needs world = parties + 1 ({cfg.parties + 1})")
    dev = ctx.device
    torch.manual_seed(cfg.seed)
    bottoms = [T.BottomModel(len(p), 2 * len(p)) for p in parts]
    top = T.TopModel(bottoms, 2)
    dims = [2 * len(p) for p in parts]
    if ctx.rank == 0:
        y = torch.tensor(Ytr.values.astype(np.float32)).to(dev)
        node = SplitNNServer(top.to(dev), list(range(1, cfg.parties + 1)), dims)
    else:
        i = ctx.rank - 1
        x = torch.tensor(Xtr[parts[i]].values.astype(np.float32)).to(dev)
        node = SplitNNParty(bottoms[i].to(dev), dims[i])
    start, prior, on_epoch = _splitnn_checkpointing(cfg, ctx, node)
    if ctx.rank == 0:
        hist = prior + node.fit(y, cfg.epochs, cfg.batch_size, start_epoch=start, on_epoch=on_epoch)
        yte = torch.tensor(Yte.values.astype(np.float32)).to(dev)
        out = node.infer(len(yte), yte)
        acc = (out.argmax(1) == yte.argmax(1)).float().mean().item()
        return {"train_loss": hist[-1][0], "train_accuracy": hist[-1][1], "test_accuracy": acc,
                "resumed_from": start or None}
    node.fit(x, cfg.epochs, cfg.batch_size, start_epoch=start, on_epoch=on_epoch)
    node.infer(torch.tensor(Xte[parts[i]].values.astype(np.float32)).to(dev))
    return {}


def _splitnn_checkpointing(cfg, ctx, node):
    """Per-rank shards (this rank's bottom or top model, its optimizer moments, its dropout RNG
    stream, the server's epoch history) through runtime/checkpoint.py. Returns (first epoch to
    run, history of the epochs already done, per-epoch hook)."""
    if not cfg.ckpt_dir:
        return 0, [], None
    from ..runtime.checkpoint import ShardedCheckpoint, load_optimizer_state, optimizer_state
    tag = f"splitnn,parties={cfg.parties},partition={cfg.partition},bs={cfg.batch_size},seed={cfg.seed}"
    ck = ShardedCheckpoint(cfg.ckpt_dir, ctx, tag=tag)
    cuda = ctx.device.type == "cuda"
    start, prior = 0, []
    got = ck.load()
    if got is not None:
        start, st = got
        for k, m in node.modules().items():
            m.load_state_dict(st["model"][k])
        load_optimizer_state(node.opt, st["opt"])
        torch.set_rng_state(st["rng"])
        if cuda:
            torch.cuda.set_rng_state(st["cuda_rng"])
        prior = [tuple(h) for h in st["hist"]]

    def save(e):
        hist = prior + [tuple(h.tolist()) for h in getattr(node, "history", [])]
        st = {"model": {k: m.state_dict() for k, m in node.modules().items()},
              "opt": optimizer_state(node.opt), "rng": torch.get_rng_state(), "hist": hist}
        if cuda:
            st["cuda_rng"] = torch.cuda.get_rng_state()
        ck.save(e, st)

    def on_epoch(e):
        if (cfg.ckpt_every and e % cfg.ckpt_every == 0) or e == cfg.epochs:
            save(e)

    return start, prior, on_epoch
