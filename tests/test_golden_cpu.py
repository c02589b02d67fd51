"""Golden-curve regression against the reference's own published outputs.

Only the heart-disease table ships with the reference (``lab/tutorial_2a/heart.csv``, read-only);
MNIST / TinyStories curves are not reproducible offline. Inits and RNG streams differ from the
reference run, so the checks are tolerance bands around the published numbers, not exact values.
Skipped when the reference CSV is not mounted (the synthetic stand-in has no published curve).
"""
import pytest
import torch

from ddl25spring_amd.data import heart as H
from ddl25spring_amd.models import tabular as T


@pytest.fixture(scope="module")
def real_heart():
    df, real = H.load_heart()
    if not real:
        pytest.skip("reference heart.csv not mounted")
    return df


@pytest.fixture(autouse=True)
def _one_thread():
    """The tabular nets are tiny: one intra-op thread runs them 5-20x faster than eight."""
    n = torch.get_num_threads()
    torch.set_num_threads(1)
    yield
    torch.set_num_threads(n)


def test_vfl_splitnn_matches_published_accuracy(real_heart):
    """lab/tutorial_2b/lab-vfl.ipynb:572-573: 4 parties (raw-column partition), 300 epochs, B=64,
    seed 42 -> test accuracy 86.76 %. That run trained with the reference's quirks (bottom models
    never optimised, Q5; zero_grad per epoch, Q6; dropout at test, Q8), reproduced by parity=True.
    Measured here: 89.2 % (seeds 43/44: 85.3 / 88.7 %); with the quirks fixed: 95.6 %."""
    X, Y = H.vfl_frame(real_heart)
    parts = H.partition_raw_columns(list(real_heart.columns), list(X.columns), 4)
    Xtr, Xte = H.row_split(X)
    Ytr, Yte = H.row_split(Y)
    accs = {}
    for parity in (True, False):
        torch.manual_seed(42)
        net = T.VFLNetwork([T.BottomModel(len(p), 2 * len(p)) for p in parts], 2, parity=parity)
        net.train_with_settings(300, 64, 4, parts, Xtr, Ytr)
        accs[parity] = float(net.test(Xte, Yte)[0])
    assert abs(accs[True] - 0.8676) < 0.05, accs
    assert accs[False] >= accs[True] - 0.01, accs


def test_vflvae_matches_published_loss_curve(real_heart):
    """lab/homework-2.ipynb:531,1030: VFL-VAE, 4 parties (balanced partition), full batch,
    Adam 1e-3: loss 114,117.9 at epoch 1 and 22,412.9 at epoch 500. Measured here: 112,131 and
    23,215 (1000 epochs: 14,497 vs 13,898.3 published)."""
    std = H.standard_frame(real_heart)
    parts = H.partition_balanced(list(std.columns), 4)
    xs = [torch.tensor(std[p].values).float() for p in parts]
    torch.manual_seed(0)
    m = T.VFLVAE([T.ClientEncoder(len(p), 8) for p in parts], T.ServerVAE(32, 48, 32, 16),
                 [T.ClientDecoder(8, len(p)) for p in parts], 8)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    curve = []
    for _ in range(500):
        opt.zero_grad()
        rc, mu, lv, lat, rcat = m(xs)
        loss = T.combined_loss(xs, rc, lat, rcat, mu, lv)
        loss.backward()
        opt.step()
        curve.append(loss.item())
    assert abs(curve[0] / 114117.9 - 1) < 0.10, curve[0]
    assert abs(curve[-1] / 22412.9 - 1) < 0.10, curve[-1]


def _vfl_parity_run(X, Y, parts, device="cpu", epochs=300):
    """One reference-style VFL run (lab/homework-2.ipynb cells 2 / 4): the reference's quirks on
    (parity=True: bottom models not optimised, zero_grad per epoch, dropout at test), B=64."""
    Xtr, Xte = H.row_split(X)
    Ytr, Yte = H.row_split(Y)
    net = T.VFLNetwork([T.BottomModel(len(p), 2 * len(p)) for p in parts], 2, parity=True)
    if device != "cpu":
        net = net.to(device)
    net.train_with_settings(epochs, 64, len(parts), parts, Xtr, Ytr)
    return float(net.test(Xte, Yte)[0])


def test_vfl_feature_permutations_match_published(real_heart):
    """lab/homework-2.ipynb:95,98,101 (cell 2): 4 parties, the 30 encoded columns permuted with
    np.random.seed(42 + i) and split 7/7/7/9, torch.manual_seed(42) ONCE before the three runs,
    300 epochs, B=64 -> 86.76 / 92.16 / 83.82 %. Bands of +-5 pp (our init / RNG streams differ).
    Measured here: 83.33 / 91.18 / 85.78 %."""
    X, Y = H.vfl_frame(real_heart)
    torch.manual_seed(42)
    accs = [_vfl_parity_run(X, Y, H.partition_random(list(X.columns), 4, 42 + i)) for i in range(3)]
    for got, want in zip(accs, (0.8676, 0.9216, 0.8382)):
        assert abs(got - want) <= 0.05, accs


def test_vfl_party_scaling_matches_published(real_heart):
    """lab/homework-2.ipynb:302,306,310,314 (cell 4): 2 / 4 / 6 / 8 parties on the balanced split of
    the 30 encoded columns (D6), torch.manual_seed(42) ONCE before the four runs -> 90.20 / 84.31 /
    83.33 / 79.90 %. Bands of +-5 pp. Measured here: 91.18 / 86.27 / 83.33 / 78.43 %."""
    X, Y = H.vfl_frame(real_heart)
    torch.manual_seed(42)
    accs = {n: _vfl_parity_run(X, Y, H.partition_balanced(list(X.columns), n)) for n in (2, 4, 6, 8)}
    for n, want in zip((2, 4, 6, 8), (0.9020, 0.8431, 0.8333, 0.7990)):
        assert abs(accs[n] - want) <= 0.05, accs


def test_vflvae_epoch_1000_matches_published(real_heart):
    """lab/homework-2.ipynb:1530: VFL-VAE loss 13,898.3 after 1,000 full-batch Adam epochs (+-10 %)."""
    std = H.standard_frame(real_heart)
    parts = H.partition_balanced(list(std.columns), 4)
    xs = [torch.tensor(std[p].values).float() for p in parts]
    torch.manual_seed(0)
    m = T.VFLVAE([T.ClientEncoder(len(p), 8) for p in parts], T.ServerVAE(32, 48, 32, 16),
                 [T.ClientDecoder(8, len(p)) for p in parts], 8)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    for _ in range(1000):
        opt.zero_grad()
        rc, mu, lv, lat, rcat = m(xs)
        loss = T.combined_loss(xs, rc, lat, rcat, mu, lv)
        loss.backward()
        opt.step()
    assert abs(loss.item() / 13898.3 - 1) < 0.10, loss.item()
