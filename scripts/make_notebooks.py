"""Generate the notebook front-end (``notebooks/*.ipynb``) — the framework's counterpart of the
reference's user surface (lab/tutorial_1a/horizontal-federated-learning.ipynb, lab/homework-1.ipynb,
lab/homework-2.ipynb, lab/tutorial_2b/lab-vfl.ipynb).

The notebooks are generated (not hand-edited JSON) so they stay in sync with the API; every code
cell runs top to bottom on a CPU in seconds with ``DDL_NOTEBOOK_QUICK=1``
(tests/test_notebooks_cpu.py) and at full size on an MI355X.

    python scripts/make_notebooks.py            # rewrites notebooks/*.ipynb
"""
from __future__ import annotations

import json
from pathlib import Path

OUT = Path(__file__).resolve().parent.parent / "notebooks"

SETUP = '''import os, sys
from pathlib import Path
# the repository root on sys.path when the notebook runs from notebooks/
ROOT = Path.cwd().parent if Path.cwd().name == "notebooks" else Path.cwd()
sys.path.insert(0, str(ROOT))
QUICK = os.environ.get("DDL_NOTEBOOK_QUICK", "0") == "1"  # tiny sizes: CI / a CPU-only machine
import matplotlib
if QUICK:
    matplotlib.use("Agg")
import matplotlib.pyplot as plt
import pandas as pd
import torch
print("device:", "cuda (MI355X)" if torch.cuda.is_available() else "cpu", "| quick:", QUICK)'''

PLOT = '''def lineplot(df, x, y, hue, title):
    fig, ax = plt.subplots(figsize=(6, 3.5))
    for name, g in df.groupby(hue, sort=False):
        ax.plot(g[x], g[y], marker="o", label=str(name))
    ax.set_xlabel(x); ax.set_ylabel(y); ax.set_title(title); ax.legend(fontsize=8)
    plt.show()'''


def md(text):
    return {"cell_type": "markdown", "metadata": {}, "source": text.strip("\n").splitlines(True)}


def code(text):
    return {"cell_type": "code", "metadata": {}, "execution_count": None, "outputs": [],
            "source": text.strip("\n").splitlines(True)}


def notebook(cells):
    return {"cells": cells, "metadata": {
        "kernelspec": {"display_name": "Python 3", "language": "python", "name": "python3"},
        "language_info": {"name": "python", "version": "3.10"}}, "nbformat": 4, "nbformat_minor": 5}


# ------------------------------------------------------------------------------ tutorial 1a
def tutorial_1a():
    return notebook([
        md('''
# Tutorial 1a — horizontal federated learning on MI355X

Counterpart of the reference's `lab/tutorial_1a/horizontal-federated-learning.ipynb`: centralized
SGD, FedSGD and FedAvg (McMahan et al., 2017) on MNIST-shaped data with the small CNN, and the
accuracy-per-round plot. The class names are the reference's
(`ddl25spring_amd.compat.hfl_complete`), but a server does not loop over per-client `nn.Module`
copies: all clients sampled in a round train *together* — their weights are one `[clients, P]`
buffer in HBM, every layer is one client-batched MFMA kernel, and a local step is replayed from a
HIP graph. MNIST is a learnable synthetic stand-in unless `DDL_DATA_ROOT` holds a torchvision copy
(nothing is downloaded).
'''),
        code(SETUP),
        code(PLOT),
        md('''
## Data and model
`configure` shrinks the data set for a quick run; `split(nr_clients, iid, seed)` returns one
`Subset` per client (IID: a seeded shuffle; non-IID: label-sorted shards, two per client).
'''),
        code('''from ddl25spring_amd.compat.hfl_complete import *  # reference names: split, MnistCnn, servers, RunResult
if QUICK:
    configure(n_train=2000, n_test=400)
N, ROUNDS = (10, 2) if QUICK else (100, 5)
subsets = split(N, True, 42)
print(len(subsets), "clients,", len(subsets[0]), "samples on client 0")
model = MnistCnn()
print("MnistCnn parameters:", model.store.P)'''),
        md('''
## The local training epoch
The reference leaves `train_epoch(model, loader, optimizer)` as an exercise. Here it is one
forward/backward/update per mini-batch of the native model — shown on a plain loader so the
notebook's building blocks stay recognisable. (Servers below never call it: they use the fused
client-batched trainer.)
'''),
        code('''import inspect
print(inspect.getsource(train_epoch))'''),
        md('## Centralized baseline, FedSGD and FedAvg'),
        code('''results = {}
results["Centralized"] = CentralizedServer(0.5, 1024, 42).run(ROUNDS)
results["FedSGD"] = FedSgdGradientServer(0.02, subsets, 0.2, 42).run(ROUNDS)
results["FedAvg"] = FedAvgServer(0.02, 200, subsets, 0.2, 2, 42).run(ROUNDS)
df = pd.concat([r.as_df() for r in results.values()], ignore_index=True)
df'''),
        code('lineplot(df, "Round", "Test accuracy", "Algorithm", "Tutorial 1a: accuracy per round")'),
        md('''
## Beyond the tutorial: the native engine
The same algorithms, Byzantine-robust aggregation (Krum / trimmed mean / coordinate median, on
client *updates*) and attacks are one constructor away in `ddl25spring_amd.fl`. With several
GPUs (`python -m ddl25spring_amd.runtime.launch -n 8 ...`) each rank trains its share of the
clients and the server state is reduced over RCCL.
'''),
        code('''from ddl25spring_amd.data.images import DeviceImageDataset, load_images
from ddl25spring_amd.data.split import split as split_idx
from ddl25spring_amd.fl.algorithms import FedAvg
from ddl25spring_amd.fl.attacks import make_attack
from ddl25spring_amd.models import mnist_cnn
dev = torch.device("cuda" if torch.cuda.is_available() else "cpu")
train = load_images("mnist", True, 2000 if QUICK else 60000)
test = load_images("mnist", False, 400 if QUICK else 10000)
parts = split_idx(N, True, 0, labels=train.labels)
rows = []
for agg in ("mean", "median", "krum"):
    fa = FedAvg(mnist_cnn, DeviceImageDataset(train, dev), parts, lr=0.05, batch_size=50,
                client_fraction=1.0, seed=0, test_data=DeviceImageDataset(test, dev), aggregator=agg,
                agg_kwargs={"f": 2}, attack=make_attack("sign_flip", [0, 1]), eval_every=0)
    for _ in range(ROUNDS):
        fa.round()
    rows.append({"aggregator": agg, "test accuracy (2 sign-flip attackers)": fa.test()})
pd.DataFrame(rows)'''),
    ])


# ------------------------------------------------------------------------------ tutorial 1a (template)
def tutorial_1a_template():
    """The exercise version of tutorial 1a: the reference template's nine `# TODO` cells
    (lab/tutorial_1a/horizontal-federated-learning.ipynb) as stubs to fill
    in, each checked against the framework's solution (compat.hfl_complete) once implemented."""
    return notebook([
        md("""
# Tutorial 1a (exercise) — horizontal federated learning

The exercise form of `tutorial_1a_horizontal_fl.ipynb`: the nine building blocks of FedSGD /
FedAvg are left as `# TODO` stubs with the reference's names and signatures. Fill them in with
plain PyTorch; the last cell runs every server whose pieces are implemented, compares the client
split with the framework's solution (`ddl25spring_amd.compat.hfl_complete`, the client-batched
native engine) and lists the pieces still missing. Data is the learnable MNIST-shaped stand-in
unless `DDL_DATA_ROOT` holds MNIST.
"""),
        code(SETUP),
        code("""import numpy as np
import torch.nn.functional as F
from torch.utils.data import DataLoader, Subset
from ddl25spring_amd.compat import hfl_complete as solution
from ddl25spring_amd.compat.hfl_complete import RunResult, configure
from ddl25spring_amd.models.torch_ref import TorchMnistCnn as MnistCnn  # a plain nn.Module CNN
if QUICK:
    configure(n_train=2000, n_test=400)
train_dataset, test_loader = solution.train_dataset, solution.test_loader
device = torch.device("cuda" if torch.cuda.is_available() else "cpu")
TODO = NotImplementedError"""),
        md("## 1. The local epoch and the client split"),
        code("""def train_epoch(model, loader, optimizer):
    # TODO: model.train(); for every (x, y) batch moved to `device`: zero_grad, forward,
    #       F.nll_loss, backward, optimizer.step()
    raise TODO("train_epoch")


def split(nr_clients, iid, seed):
    # TODO: rng = np.random.default_rng(seed); IID: rng.permutation of all indices cut into
    #       nr_clients parts; non-IID: sort by label, cut into 2 * nr_clients shards, shuffle the
    #       shard ids, give every client two shards. Return [Subset(train_dataset, idx), ...]
    raise TODO("split")"""),
        md("## 2. Clients and servers"),
        code("""class Client:
    def __init__(self, client_data, batch_size):
        self.model = MnistCnn().to(device)
        self.generator = torch.Generator()
        self.loader = DataLoader(client_data, batch_size=batch_size, shuffle=True, generator=self.generator)

    def update(self, weights, seed):
        raise NotImplementedError


class Server:
    def __init__(self, lr, batch_size, seed):
        self.lr, self.batch_size, self.seed = lr, batch_size, seed
        torch.manual_seed(seed)
        self.model = MnistCnn().to(device)

    def run(self, nr_rounds):
        raise NotImplementedError

    def test(self):
        # TODO: eval mode, no_grad, one pass over test_loader, argmax, return 100 * correct / total
        raise TODO("Server.test")


class CentralizedServer(Server):
    def __init__(self, lr, batch_size, seed):
        super().__init__(lr, batch_size, seed)
        self.optimizer = torch.optim.SGD(self.model.parameters(), lr=lr)
        self.generator = torch.Generator()
        self.loader = DataLoader(train_dataset, batch_size=batch_size, shuffle=True, generator=self.generator)

    def run(self, nr_rounds):
        # TODO: per round (one epoch): generator.manual_seed(seed + epoch + 1), train_epoch, then
        #       append wall time, message count 0 and self.test() to
        #       RunResult("Centralized", 1, 1, batch_size, 1, lr, seed)
        raise TODO("CentralizedServer.run")


class DecentralizedServer(Server):
    def __init__(self, lr, batch_size, client_subsets, client_fraction, seed):
        super().__init__(lr, batch_size, seed)
        self.nr_clients = len(client_subsets)
        self.client_fraction = client_fraction
        self.client_sample_counts = [len(s) for s in client_subsets]
        # TODO: self.nr_clients_per_round = max(1, round(client_fraction * nr_clients));
        #       self.rng = np.random.default_rng(seed)
        raise TODO("DecentralizedServer.__init__")


class GradientClient(Client):
    def __init__(self, client_data):
        super().__init__(client_data, len(client_data))

    def update(self, weights, seed):
        # TODO: copy `weights` into the model, zero the grads, one full-batch forward/backward
        #       (nll_loss), return [p.grad.detach().cpu().clone() for p in parameters]
        raise TODO("GradientClient.update")


class FedSgdGradientServer(DecentralizedServer):
    def __init__(self, lr, client_subsets, client_fraction, seed):
        super().__init__(lr, -1, client_subsets, client_fraction, seed)
        self.clients = [GradientClient(s) for s in client_subsets]
        self.optimizer = torch.optim.SGD(self.model.parameters(), lr=lr)

    def run(self, nr_rounds):
        # TODO: per round: sample K clients without replacement (self.rng), client seed
        #       seed + idx + 1 + round * K, weight each client's gradients by n_k / sum(n_k), sum
        #       them, set .grad and take one SGD step; message_count 2 * (round + 1) * K
        raise TODO("FedSgdGradientServer.run")


class WeightClient(Client):
    def __init__(self, client_data, lr, batch_size, nr_epochs):
        super().__init__(client_data, batch_size)
        self.optimizer = torch.optim.SGD(self.model.parameters(), lr=lr)
        self.nr_epochs = nr_epochs

    def update(self, weights, seed):
        # TODO: copy `weights` in, generator.manual_seed(seed), nr_epochs x train_epoch,
        #       return [p.detach().cpu().clone() for p in parameters]
        raise TODO("WeightClient.update")


class FedAvgServer(DecentralizedServer):
    def __init__(self, lr, batch_size, client_subsets, client_fraction, nr_local_epochs, seed):
        super().__init__(lr, batch_size, client_subsets, client_fraction, seed)
        self.clients = [WeightClient(s, lr, batch_size, nr_local_epochs) for s in client_subsets]
        self.nr_local_epochs = nr_local_epochs

    def run(self, nr_rounds):
        # TODO: as FedSGD, but average the returned WEIGHTS (n_k-weighted) into the server model
        raise TODO("FedAvgServer.run")"""),
        md("## 3. Run what is implemented"),
        code("""N, ROUNDS = (10, 1) if QUICK else (100, 5)
status = []


def attempt(name, fn):
    try:
        out = fn()
        status.append((name, "implemented"))
        return out
    except NotImplementedError as e:
        status.append((name, f"TODO ({e})"))
        return None


subsets = attempt("split", lambda: split(N, True, 42))
ref = solution.split(N, True, 42)
if subsets is not None:
    assert [len(s) for s in subsets] == [len(s) for s in ref], "split: client sizes differ from the solution"
else:
    subsets = [Subset(train_dataset, list(s.indices)) for s in ref]
for name, make in [("CentralizedServer", lambda: CentralizedServer(0.5, 1024, 42)),
                   ("FedSgdGradientServer", lambda: FedSgdGradientServer(0.02, subsets, 0.2, 42)),
                   ("FedAvgServer", lambda: FedAvgServer(0.02, 200, subsets, 0.2, 1, 42))]:
    res = attempt(name, lambda: make().run(ROUNDS))
    if res is not None:
        print(name, "test accuracy per round:", res.test_accuracy)
pd.DataFrame(status, columns=["piece", "status"])"""),
    ])


# ------------------------------------------------------------------------------ homework 1
def homework_1():
    return notebook([
        md('''
# Homework 1 — FedSGD vs FedAvg, and data / pipeline parallelism

Counterpart of the reference's `lab/homework-1.ipynb`. Part A runs the federated-learning
experiments (defaults: N = 100 clients, lr = 0.01, C = 0.1, E = 1, B = 100, 10 rounds, IID,
seed 10). Part B trains the tiny LLaMA with a micro-batched pipeline and with a data x pipeline
grid — one process per rank (one per GPU over RCCL on an MI355X node, gloo ranks on a CPU).
'''),
        code(SETUP),
        code(PLOT),
        code('''from ddl25spring_amd.compat.hfl_complete import *
if QUICK:
    configure(n_train=2000, n_test=400)
n, lr, c, e, b, seed = (10, 0.01, 0.1, 1, 100, 10) if QUICK else (100, 0.01, 0.1, 1, 100, 10)
R5, R10, R15 = (2, 2, 2) if QUICK else (5, 10, 15)'''),
        md('''
## A1 — FedSGD exchanging weights instead of gradients
With one local step on the whole local data set (E = 1, B = inf), a client that returns its
updated *weights* and a client that returns its *gradient* produce the same server update:
`w - lr * mean_k g_k = mean_k (w - lr * g_k)`. The two runs agree round by round.
'''),
        code('''sub = split(n, True, seed)
g = FedSgdGradientServer(lr, sub, 0.5, seed).run(R5).as_df()
w = FedSgdWeightServer(lr, sub, 0.5, seed).run(R5).as_df()
pd.DataFrame({"Round": g["Round"], "gradients": g["Test accuracy"], "weights": w["Test accuracy"],
              "difference": w["Test accuracy"] - g["Test accuracy"]})'''),
        md('## A2 — number of clients and client fraction'),
        code('''rows = []
for nn_ in ((4, 10) if QUICK else (10, 50, 100)):
    s = split(nn_, True, seed)
    for name, srv in (("FedSGD", FedSgdGradientServer(lr, s, c, seed)),
                      ("FedAvg", FedAvgServer(lr, b, s, c, e, seed))):
        r = srv.run(R10).as_df().iloc[-1]
        rows.append({"N": nn_, "C": c, "Algorithm": name, "Test accuracy": r["Test accuracy"],
                     "Message count": r["Message count"]})
s = split(n, True, seed)
for cc in (0.01, 0.1, 0.2):
    for name, srv in (("FedSGD", FedSgdGradientServer(lr, s, cc, seed)),
                      ("FedAvg", FedAvgServer(lr, b, s, cc, e, seed))):
        r = srv.run(R10).as_df().iloc[-1]
        rows.append({"N": n, "C": cc, "Algorithm": name, "Test accuracy": r["Test accuracy"],
                     "Message count": r["Message count"]})
pd.DataFrame(rows)'''),
        md('## A3 — local epochs, IID vs non-IID'),
        code('''s = split(n, True, seed)
frames = []
for ep in (1, 2, 4):
    d = FedAvgServer(lr, b, s, c, ep, seed).run(R10).as_df()
    d["Algorithm"] = f"FedAvg E={ep}"
    frames.append(d)
d = FedSgdGradientServer(lr, s, c, seed).run(R10).as_df(); d["Algorithm"] = "FedSGD"
frames.append(d)
lineplot(pd.concat(frames), "Round", "Test accuracy", "Algorithm", "Local epochs")'''),
        code('''frames = []
for iid in (True, False):
    s = split(n, iid, seed)
    for name, srv in (("FedSGD", FedSgdGradientServer(lr, s, c, seed)),
                      ("FedAvg", FedAvgServer(lr, b, s, c, e, seed))):
        d = srv.run(R15).as_df()
        d["Algorithm"] = f"{name} {'IID' if iid else 'non-IID'}"
        frames.append(d)
lineplot(pd.concat(frames), "Round", "Test accuracy", "Algorithm", "IID vs non-IID")'''),
        md('''
## B1 — micro-batched pipeline parallelism
Three pipeline stages (two LLaMA blocks each), batch 3 split into 3 micro-batches, GPipe schedule
(all forwards, then all backwards). The launcher starts one process per stage; activations and
their gradients move over RCCL point-to-point (gloo on a CPU). Every schedule is checked for
send/recv deadlocks before it runs.
'''),
        code('''import subprocess
TINY = ["--dmodel", "48", "--num-heads", "2", "--n-layers", "3", "--ctx-size", "32",
        "--vocab-size", "512", "--iters", "3", "--log-every", "1"] if QUICK else ["--iters", "100"]
DEV = ["--device", "cpu"] if QUICK or not torch.cuda.is_available() else []

def llm(world, *args):
    cmd = [sys.executable, "-m", "ddl25spring_amd.runtime.launch", "-n", str(world), "--timeout", "1800",
           "-m", "ddl25spring_amd", *DEV, "llm", *args, *TINY]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True)
    print(out.stdout[-2000:]); assert out.returncode == 0, out.stderr[-3000:]

llm(3, "--pp", "3", "--batch-size", "3", "--micro-batches", "3", "--schedule", "gpipe")'''),
        md('''
## B2 — data and pipeline parallelism together
Two pipelines of three stages (6 ranks), 1F1B schedule. The data-parallel groups (stage s of
every pipeline) are created collectively on every rank, and their gradients are all-reduced in
buckets overlapped with the backward pass.
'''),
        code('llm(6, "--dp", "2", "--pp", "3", "--batch-size", "3", "--micro-batches", "3", "--schedule", "1f1b")'),
    ])


# ------------------------------------------------------------------------------ lab VFL
def lab_vfl():
    return notebook([
        md('''
# Vertical federated learning — split learning

Counterpart of the reference's `lab/tutorial_2b/lab-vfl.ipynb`. Parties hold different *columns*
of the same rows (the heart-disease table); each trains a bottom model on its columns, and the
label holder trains a top model on the concatenated cut-layer activations. Only activations and
their gradients cross party boundaries.
'''),
        code(SETUP),
        code(PLOT),
        code('''import numpy as np
from ddl25spring_amd.compat import vfl as V
from ddl25spring_amd.models.tabular import BottomModel, TopModel, VFLNetwork
df, real = V.load_heart()
print("heart.csv" if real else "synthetic table with the heart.csv schema", df.shape)
X, Y = V.vfl_frame(df)          # one-hot encoded features, one-hot target
feats = V.partition_raw_columns(list(df.columns), list(X.columns), 4)
print("features per party:", [len(f) for f in feats])
Xtr, Xte = V.row_split(X); Ytr, Yte = V.row_split(Y)'''),
        md('''
## Bottom models, top model, and the joint network
`VFLNetwork` keeps the reference's training loop shape (`train_with_settings`, `test`). Its
defaults fix three quirks of the reference (bottom models never optimised, gradients accumulated
over an epoch, dropout active at test); `parity=True` restores them. On the GPU every linear is
an MFMA kernel with the activation fused, the optimizer is one fused AdamW launch over a flat
parameter buffer, and loss / accuracy are accumulated on the device (no per-batch host sync).
'''),
        code('''torch.manual_seed(42); np.random.seed(42)
dev = "cuda" if torch.cuda.is_available() else "cpu"
net = VFLNetwork([BottomModel(len(f), 2 * len(f)) for f in feats], 2).to(dev)
EPOCHS = 5 if QUICK else 300
hist = net.train_with_settings(EPOCHS, 64, 4, feats, Xtr, Ytr)
acc, loss = net.test(Xte, Yte)
print(f"test accuracy {100 * float(acc):.2f} %, test loss {float(loss):.3f}")
curve = pd.DataFrame({"Epoch": range(1, EPOCHS + 1), "Loss": [h[0] for h in hist], "Run": "split-NN"})
lineplot(curve, "Epoch", "Loss", "Run", "split-NN training loss")'''),
        md('''
## One party per process
The same split-NN with every party in its own process (rank 0 = label holder); cut-layer tensors
move with grouped point-to-point sends. `--ckpt-dir` checkpoints every rank's shard so a killed
run resumes exactly where it stopped.
'''),
        code('''import subprocess
DEV = ["--device", "cpu"] if QUICK or not torch.cuda.is_available() else []
cmd = [sys.executable, "-m", "ddl25spring_amd.runtime.launch", "-n", "3", "--timeout", "600",
       "-m", "ddl25spring_amd", *DEV, "vfl", "--task", "splitnn", "--parties", "2",
       "--partition", "balanced", "--epochs", str(EPOCHS)]
out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True)
print(out.stdout[-1500:]); assert out.returncode == 0, out.stderr[-3000:]'''),
    ])


# ------------------------------------------------------------------------------ homework 2
def homework_2():
    return notebook([
        md('''
# Homework 2 — vertical FL and generative modeling

Counterpart of the reference's `lab/homework-2.ipynb`: (1) how the assignment of features to
parties changes split-NN accuracy, (2) how the number of parties does, and (3) a VFL variational
autoencoder whose parties encode their columns locally and a server VAE models the joint latent.
'''),
        code(SETUP),
        code(PLOT),
        code('''import numpy as np
from ddl25spring_amd.compat import vfl as V
from ddl25spring_amd.models.tabular import BottomModel, VFLNetwork
df, _ = V.load_heart()
X, Y = V.vfl_frame(df); cols = list(X.columns)
Xtr, Xte = V.row_split(X); Ytr, Yte = V.row_split(Y)
EPOCHS = 5 if QUICK else 300
dev = "cuda" if torch.cuda.is_available() else "cpu"

def run(feats, seed=42):
    torch.manual_seed(seed); np.random.seed(seed)
    net = VFLNetwork([BottomModel(len(f), 2 * len(f)) for f in feats], 2).to(dev)
    hist = net.train_with_settings(EPOCHS, 64, len(feats), feats, Xtr, Ytr)
    acc, loss = net.test(Xte, Yte)
    return hist, 100 * float(acc)'''),
        md('## Exercise 1 — random feature permutations (4 parties)'),
        code('''rows, curves = [], []
for seed in (42, 43, 44):
    hist, acc = run(V.partition_random(cols, 4, seed))
    rows.append({"permutation seed": seed, "test accuracy %": acc})
    curves.append(pd.DataFrame({"Epoch": range(1, EPOCHS + 1), "Loss": [h[0] for h in hist],
                                "Run": f"seed {seed}"}))
lineplot(pd.concat(curves), "Epoch", "Loss", "Run", "Feature permutations")
pd.DataFrame(rows)'''),
        md('## Exercise 2 — number of parties (balanced partition)'),
        code('''rows = []
for n in (2, 4, 6, 8):
    _, acc = run(V.partition_balanced(cols, n))
    rows.append({"parties": n, "test accuracy %": acc})
pd.DataFrame(rows)'''),
        md('''
## Exercise 3 — VFL-VAE
Four parties with 8-dimensional client latents, a server VAE (latent 16) over their
concatenation, and per-party decoders; full-batch Adam on the standardised table.
'''),
        code('''from ddl25spring_amd.compat.exercise_3 import ClientDecoder, ClientEncoder, ServerVAE, VFLVAE, combined_loss
from ddl25spring_amd.data import heart as H
from ddl25spring_amd.optim import make_adam
torch.manual_seed(42)
std = H.standard_frame(df)
parts = H.partition_balanced(list(std.columns), 4)
xs = [torch.tensor(std[p].values).float().to(dev) for p in parts]
m = VFLVAE([ClientEncoder(len(p), 8) for p in parts], ServerVAE(4 * 8, 48, 32, 16),
           [ClientDecoder(8, len(p)) for p in parts], 8).to(dev)
opt = make_adam(m.parameters(), lr=1e-3)
losses = []
for _ in range(10 if QUICK else 1000):
    opt.zero_grad()
    rc, mu, lv, lat, rcat = m(xs)
    loss = combined_loss(xs, rc, lat, rcat, mu, lv)
    loss.backward(); opt.step()
    losses.append(loss.detach())
losses = torch.stack(losses).tolist()
curve = pd.DataFrame({"Epoch": range(1, len(losses) + 1), "Loss": losses, "Run": "VFL-VAE"})
lineplot(curve, "Epoch", "Loss", "Run", "VFL-VAE loss")
curve.iloc[[0, len(curve) // 2, -1]]'''),
    ])


NOTEBOOKS = {
    "tutorial_1a_horizontal_fl.ipynb": tutorial_1a,
    "tutorial_1a_horizontal_fl_template.ipynb": tutorial_1a_template,
    "homework_1.ipynb": homework_1,
    "lab_vfl.ipynb": lab_vfl,
    "homework_2.ipynb": homework_2,
}


def main():
    OUT.mkdir(exist_ok=True)
    for name, fn in NOTEBOOKS.items():
        (OUT / name).write_text(json.dumps(fn(), indent=1) + "\n")
        print("wrote", OUT / name)


if __name__ == "__main__":
    main()
