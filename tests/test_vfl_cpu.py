"""Heart-disease data recipes, tabular nets (centralized / VAE / split-NN / VFL-VAE) and the
distributed one-party-per-rank VFL runtime (gloo) vs its single-process equivalent."""
import os
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ddl25spring_amd.data import heart as H
from ddl25spring_amd.models import tabular as T
from ddl25spring_amd.optim import FlatAdam, FlatAdamW


@pytest.fixture(scope="module")
def heart():
    df, real = H.load_heart()
    return df, real


def test_heart_schema_and_partitions(heart):
    df, real = heart
    assert list(df.columns) == H.COLUMNS and len(df) == 1025
    X, Y = H.vfl_frame(df)
    assert X.shape[1] == 30 and Y.shape[1] == 2
    parts = H.partition_raw_columns(list(df.columns), list(X.columns), 4)
    assert [len(p) for p in parts] == [7, 4, 6, 13]
    assert sorted(sum(parts, [])) == sorted(X.columns)
    rnd = H.partition_random(list(X.columns), 4, 42)
    assert [len(p) for p in rnd] == [7, 7, 7, 9] and sorted(sum(rnd, [])) == sorted(X.columns)
    std = H.standard_frame(df)
    assert std.shape[1] == 31
    assert [len(p) for p in H.partition_balanced(list(std.columns), 4)] == [8, 8, 8, 7]
    tr, te = H.row_split(X)
    assert (len(tr), len(te)) == (821, 204)
    Xtr, Xte, ytr, yte = H.centralized_split(df, seed=0)
    assert Xtr.shape == (820, 30) and Xte.shape == (205, 30)
    assert Xtr.min() >= 0 and Xtr.max() <= 1


def test_centralized_keeps_deep_copy_of_best(heart):
    df, real = heart
    torch.manual_seed(42)
    Xtr, Xte, ytr, yte = [torch.tensor(a) for a in H.centralized_split(df, seed=42)]
    net = T.HeartDiseaseNN()
    best, hist = T.train_centralized(net, Xtr, ytr.long(), Xte, yte.long(), epochs=49)
    assert best == max(a for _, a in hist)
    net.eval()
    with torch.no_grad():
        acc = (net(Xte).argmax(1) == yte).float().mean().item()
    assert acc == pytest.approx(best)  # restored weights ARE the best epoch's
    assert best > 0.75


def test_vfl_splitnn_trains_and_parity_flags(heart):
    df, _ = heart
    X, Y = H.vfl_frame(df)
    parts = H.partition_raw_columns(list(df.columns), list(X.columns), 4)
    Xtr, Xte = H.row_split(X)
    Ytr, Yte = H.row_split(Y)
    torch.manual_seed(42)
    net = T.VFLNetwork([T.BottomModel(len(p), 2 * len(p)) for p in parts], 2)
    hist = net.train_with_settings(40, 64, 4, parts, Xtr, Ytr)
    acc, loss = net.test(Xte, Yte)
    assert hist[-1][0] < hist[0][0] and acc > 0.7
    # parity mode: bottom models are NOT registered -> never optimised (reference quirk Q5)
    torch.manual_seed(42)
    bottoms = [T.BottomModel(len(p), 2 * len(p)) for p in parts]
    before = [p.detach().clone() for b in bottoms for p in b.parameters()]
    quirky = T.VFLNetwork(bottoms, 2, parity=True)
    quirky.train_with_settings(2, 64, 4, parts, Xtr, Ytr)
    after = [p.detach() for b in bottoms for p in b.parameters()]
    assert all(torch.equal(a, b) for a, b in zip(before, after))


def test_tabular_vae_and_sampling(heart):
    df, _ = heart
    Xtr, Xte, ytr, yte = H.centralized_split(df, scaler="standard", seed=42)
    real = torch.cat([torch.tensor(Xtr), torch.tensor(ytr).float().view(-1, 1)], 1)
    torch.manual_seed(0)
    vae = T.Autoencoder(real.shape[1], 48, 32, 16)
    opt = torch.optim.Adam(vae.parameters(), lr=1e-3)
    losses = vae.train_with_settings(8, 64, real, opt, T.customLoss())
    assert losses[-1] < losses[0]
    _, mu, logvar = vae(real)
    syn = vae.sample(len(real), mu.shape[1], logvar, mu)
    assert syn.shape == real.shape and set(np.unique(syn[:, -1])) <= {0.0, 1.0}


def test_vflvae_loss_decreases(heart):
    df, _ = heart
    std = H.standard_frame(df)
    parts = H.partition_balanced(list(std.columns), 4)
    xs = [torch.tensor(std[p].values).float() for p in parts]
    torch.manual_seed(0)
    m = T.VFLVAE([T.ClientEncoder(len(p), 8) for p in parts], T.ServerVAE(32, 48, 32, 16),
                 [T.ClientDecoder(8, len(p)) for p in parts], 8)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    ls = []
    for _ in range(30):
        opt.zero_grad()
        rc, mu, lv, lat, rcat = m(xs)
        loss = T.combined_loss(xs, rc, lat, rcat, mu, lv)
        loss.backward()
        opt.step()
        ls.append(loss.item())
    assert ls[-1] < 0.8 * ls[0]


@pytest.mark.parametrize("decoupled", [False, True])
def test_flat_adam_matches_torch(decoupled):
    torch.manual_seed(0)
    shapes = [(64, 30), (64,), (7, 3, 5)]
    a = [torch.nn.Parameter(torch.randn(s)) for s in shapes]
    b = [torch.nn.Parameter(p.detach().clone()) for p in a]
    tgt = [torch.randn(s) for s in shapes]
    oa = (FlatAdamW if decoupled else FlatAdam)(a, lr=1e-2, weight_decay=0.05)
    ob = (torch.optim.AdamW if decoupled else torch.optim.Adam)(b, lr=1e-2, weight_decay=0.05)
    for _ in range(10):
        for ps, o in ((a, oa), (b, ob)):
            o.zero_grad()
            sum(((p - t) ** 2).sum() for p, t in zip(ps, tgt)).backward()
            o.step()
    for pa, pb in zip(a, b):
        assert torch.allclose(pa, pb, atol=1e-6)


# ------------------------------------------------------------------ distributed (gloo, 3 ranks)
DIMS = [5, 7]
N, BS, EPOCHS = 40, 16, 3


def _splitnn_models():
    torch.manual_seed(7)
    bottoms = [T.BottomModel(d, 2 * d) for d in DIMS]
    top = T.TopModel(bottoms, 2)
    for m in bottoms + [top]:
        m.dropout.p = 0.0
    g = torch.Generator().manual_seed(3)
    xs = [torch.randn(N, d, generator=g) for d in DIMS]
    y = torch.nn.functional.one_hot(torch.randint(0, 2, (N,), generator=g), 2).float()
    return bottoms, top, xs, y


def _vae_models():
    torch.manual_seed(11)
    encs = [T.ClientEncoder(d, 4) for d in DIMS]
    decs = [T.ClientDecoder(4, d) for d in DIMS]
    vae = T.ServerVAE(8, 16, 12, 6)
    g = torch.Generator().manual_seed(5)
    xs = [torch.randn(N, d, generator=g) for d in DIMS]
    return encs, decs, vae, xs


def _vfl_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    # one intra-op thread on both sides: Adam turns float-reduction-order noise on (near-)zero
    # gradients into full +-lr steps, so the reductions must run in the same order
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ddl25spring_amd.vfl import SplitNNParty, SplitNNServer, VAEParty, VAEServer
    bottoms, top, xs, y = _splitnn_models()
    parties = [1, 2]
    if rank == 0:
        SplitNNServer(top, parties, [2 * d for d in DIMS]).fit(y, EPOCHS, BS)
        res = [p.detach() for p in top.parameters()]
    else:
        SplitNNParty(bottoms[rank - 1], 2 * DIMS[rank - 1]).fit(xs[rank - 1], EPOCHS, BS)
        res = [p.detach() for p in bottoms[rank - 1].parameters()]
    encs, decs, vae, vx = _vae_models()
    torch.manual_seed(99)  # server-side reparameterisation noise
    node = VAEServer(vae, parties, 4) if rank == 0 else VAEParty(encs[rank - 1], decs[rank - 1], 4)
    for _ in range(4):
        if rank == 0:
            loss = node.train_step(N, vx[0])
        else:
            node.train_step(vx[rank - 1])
    if rank == 0:
        vres = [p.detach() for p in vae.parameters()] + [loss.reshape(1)]
    else:
        vres = [p.detach() for p in encs[rank - 1].parameters()] + \
               [p.detach() for p in decs[rank - 1].parameters()]
    torch.save({"split": res, "vae": vres}, os.path.join(out_dir, f"r{rank}.pt"))
    dist.destroy_process_group()


def test_distributed_vfl_matches_single_process():
    nthreads = torch.get_num_threads()
    torch.set_num_threads(1)
    try:
        _check_distributed_vfl()
    finally:
        torch.set_num_threads(nthreads)


def _check_distributed_vfl():
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_vfl_worker, args=(3, 29877, d), nprocs=3, join=True)
        res = [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True) for r in range(3)]
    # single-process split-NN, one AdamW over everything (= per-party AdamW: Adam is per-parameter)
    bottoms, top, xs, y = _splitnn_models()
    params = [p for m in bottoms + [top] for p in m.parameters()]
    opt = torch.optim.AdamW(params)
    crit = torch.nn.CrossEntropyLoss()
    for _ in range(EPOCHS):
        for b in range(0, N, BS):
            opt.zero_grad()
            crit(top([m(x[b:b + BS]) for m, x in zip(bottoms, xs)]), y[b:b + BS]).backward()
            opt.step()
    for got, want in zip(res[0]["split"], top.parameters()):
        assert torch.allclose(got, want, atol=1e-5)
    for r in (1, 2):
        for got, want in zip(res[r]["split"], bottoms[r - 1].parameters()):
            assert torch.allclose(got, want, atol=1e-5)
    # single-process VFL-VAE
    encs, decs, vae, vx = _vae_models()
    model = T.VFLVAE(encs, vae, decs, 4)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    torch.manual_seed(99)
    for _ in range(4):
        opt.zero_grad()
        rc, mu, lv, lat, rcat = model(vx)
        loss = T.combined_loss(vx, rc, lat, rcat, mu, lv)
        loss.backward()
        opt.step()
    got = res[0]["vae"]
    assert abs(got[-1].item() - loss.item()) < 1e-3 * abs(loss.item())
    for g, w in zip(got[:-1], vae.parameters()):
        assert torch.allclose(g, w, atol=1e-5)
    for r in (1, 2):
        want = list(encs[r - 1].parameters()) + list(decs[r - 1].parameters())
        for g, w in zip(res[r]["vae"], want):
            assert torch.allclose(g, w, atol=1e-5)


def _active_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    # one intra-op thread on both sides: Adam turns float-reduction-order noise on (near-)zero
    # gradients into full +-lr steps, so the reductions must run in the same order
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ddl25spring_amd.vfl import SplitNNParty, SplitNNServer
    bottoms, top, xs, y = _splitnn_models()
    if rank == 0:  # active party: labels + feature block 0
        SplitNNServer(top, [1], [2 * DIMS[1]], local_bottom=bottoms[0]).fit(y, EPOCHS, BS, x_local=xs[0])
        res = [p.detach() for p in list(top.parameters()) + list(bottoms[0].parameters())]
    else:
        SplitNNParty(bottoms[1], 2 * DIMS[1]).fit(xs[1], EPOCHS, BS)
        res = [p.detach() for p in bottoms[1].parameters()]
    torch.save(res, os.path.join(out_dir, f"r{rank}.pt"))
    dist.destroy_process_group()


def test_two_party_active_passive_matches_single_process():
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_active_worker, args=(2, 29879, d), nprocs=2, join=True)
        r0 = torch.load(os.path.join(d, "r0.pt"), weights_only=True)
        r1 = torch.load(os.path.join(d, "r1.pt"), weights_only=True)
    bottoms, top, xs, y = _splitnn_models()
    opt = torch.optim.AdamW([p for m in bottoms + [top] for p in m.parameters()])
    crit = torch.nn.CrossEntropyLoss()
    for _ in range(EPOCHS):
        for b in range(0, N, BS):
            opt.zero_grad()
            crit(top([m(x[b:b + BS]) for m, x in zip(bottoms, xs)]), y[b:b + BS]).backward()
            opt.step()
    want0 = list(top.parameters()) + list(bottoms[0].parameters())
    assert all(torch.allclose(g, w, atol=1e-5) for g, w in zip(r0, want0))
    assert all(torch.allclose(g, w, atol=1e-5) for g, w in zip(r1, bottoms[1].parameters()))
