"""Drop-in module with the public names of reference ``lab/tutorial_1a/hfl_complete.py``.

Notebook code written against the reference keeps working::

    from ddl25spring_amd.compat.hfl_complete import *
    subsets = split(100, True, 10)
    result = FedAvgServer(0.01, 100, subsets, 0.1, 1, 10).run(10)
    result.as_df()

but every server runs on the MI355X engine: all sampled clients of a round train together
(client-batched kernels, weights resident in HBM, HIP-graph-captured steps) instead of the
reference's sequential per-client ``nn.Module`` loop with host round-trips.

Parity kept on purpose (reference line numbers):
  * init: ``torch.manual_seed(seed)`` then the MnistCnn architecture (:165-166) — weights are
    built by the same torch initialisers and imported, so round-0 weights are identical;
  * client sampling ``default_rng(seed).choice`` (:229,278), client shuffles
    ``torch.randperm`` with ``Generator().manual_seed(seed + idx + 1 + round*K)`` (:289,327) —
    the ``planner="torch"`` path reproduces ``DataLoader(shuffle=True, generator=...)``;
  * ``RunResult`` columns, message counts ``2*(round+1)*K`` (:309), accuracy in % (:183).
Differences: compute is bf16 on MFMA with fp32 master weights (the reference is fp32), dropout
masks come from a counter-based Philox stream, and MNIST is synthetic unless ``DDL_DATA_ROOT``
holds a torchvision copy (nothing is downloaded, nothing happens at import — SURVEY Q11).
"""
from __future__ import annotations

from pathlib import Path
from typing import cast

import numpy as np
import torch
from torch.utils.data import Subset

from ..data.images import SHAPES, DeviceImageDataset, load_images
from ..data.split import split as _split_indices
from ..fl.algorithms import FedAvg, FedSGD, FedSgdWeight
from ..fl.local import LocalTrainer
from ..fl.result import ETA, RunResult  # noqa: F401  (re-exported)
from ..models import convert
from ..models.torch_ref import TorchMnistCnn
from ..models.zoo import mnist_cnn, mnist_cnn_mapping
from ..ops import functional as Fn
from ..runtime import dist as rdist

data_path = Path(__file__).resolve().parent.parent.parent / "data"

if torch.cuda.is_available():
    device = torch.device("cuda")
else:
    device = torch.device("cpu")

MEAN, STD = SHAPES["mnist"][6][0], SHAPES["mnist"][7][0]


class transform:  # noqa: N801 - mirrors the reference's module-level `transform`
    """ToTensor + Normalize((0.1307,), (0.3081,)) as a callable on uint8 HxW(x1) arrays."""

    def __new__(cls, img):
        t = torch.as_tensor(np.asarray(img), dtype=torch.float32) / 255.0
        if t.dim() == 3:
            t = t.permute(2, 0, 1)
        else:
            t = t.unsqueeze(0)
        return (t - MEAN) / STD


class _ImageDataset(torch.utils.data.Dataset):
    """torchvision-like dataset view (uint8 arrays in host memory, lazily created)."""

    def __init__(self, arrays):
        self.arrays = arrays
        self.targets = torch.as_tensor(arrays.labels)
        self.data = arrays.images

    def __len__(self):
        return len(self.arrays)

    def __getitem__(self, i):
        return transform(self.arrays.images[i]), int(self.arrays.labels[i])


_STATE: dict = {"n_train": None, "n_test": None}


def configure(n_train: int | None = None, n_test: int | None = None):
    """Shrink the (synthetic) MNIST used by this module — for quick experiments and CI."""
    _STATE.update(n_train=n_train, n_test=n_test)
    for k in ("train_arrays", "test_arrays", "dev_train", "dev_test", "train_dataset"):
        _STATE.pop(k, None)


def _arrays(train: bool):
    key = "train_arrays" if train else "test_arrays"
    if key not in _STATE:
        _STATE[key] = load_images("mnist", train=train, n=_STATE["n_train" if train else "n_test"])
    return _STATE[key]


def _device_data(train: bool) -> DeviceImageDataset:
    key = "dev_train" if train else "dev_test"
    if key not in _STATE:
        _STATE[key] = DeviceImageDataset(_arrays(train), device)
    return _STATE[key]


class _LazyTestLoader:
    """One batch of the whole test set, like DataLoader(batch_size=10000, shuffle=False)."""

    @property
    def dataset(self):
        return _ImageDataset(_arrays(False))

    def __iter__(self):
        a = _arrays(False)
        x = torch.stack([transform(im) for im in a.images])
        yield x, torch.as_tensor(a.labels)

    def __len__(self):
        return 1


def __getattr__(name):  # lazy module attributes (no download / generation at import)
    if name == "train_dataset":
        if "train_dataset" not in _STATE:
            _STATE["train_dataset"] = _ImageDataset(_arrays(True))
        return _STATE["train_dataset"]
    if name == "test_loader":
        return _LazyTestLoader()
    raise AttributeError(name)


# ------------------------------------------------------------------------------------- model
def MnistCnn(groups: int = 1):  # noqa: N802 - reference class name
    """Native MnistCnn initialised exactly like ``torch.manual_seed(s); MnistCnn()`` would be."""
    tm = TorchMnistCnn()  # consumes the global torch RNG exactly like the reference constructor
    net = mnist_cnn(groups).to(device)
    convert.import_torch(net, tm, mnist_cnn_mapping())
    return net


def _init_like_reference(seed: int):
    def f(net):
        torch.manual_seed(seed)
        convert.import_torch(net, TorchMnistCnn(), mnist_cnn_mapping())
    return f


def train_epoch(model, loader, optimizer) -> None:
    """One epoch over ``loader`` (reference :71-80) on the native fused path."""
    model.train()
    for data, target in loader:
        x = model.prepare_input(data.to(model.device))
        model.zero_grad()
        model.train_step(x, target.to(model.device).reshape(1, -1).to(torch.int32))
        optimizer.step()


def split(nr_clients: int, iid: bool, seed: int) -> list[Subset]:
    ds = __getattr__("train_dataset")
    parts = _split_indices(nr_clients, iid, seed, labels=ds.targets.numpy())
    return [Subset(ds, cast(list, p.tolist())) for p in parts]


def _indices(subsets) -> list[np.ndarray]:
    return [np.asarray(s.indices, dtype=np.int64) for s in subsets]


# ------------------------------------------------------------------------------- client ABCs
class Client:
    """A client holding its own data (reference :145-155). ``update`` runs on a G=1 native net."""

    def __init__(self, client_data: Subset, batch_size: int) -> None:
        self.client_data = client_data
        self.batch_size = batch_size
        self.model = mnist_cnn(1).to(device)
        self.generator = torch.Generator()

    def _load(self, weights):
        st = self.model.store
        flat = torch.cat([w.reshape(-1).float() for w in weights]).to(st.device) \
            if isinstance(weights, (list, tuple)) else weights.to(st.device)
        st.data[0, :flat.numel()].copy_(flat)
        st.sync_shadow()

    def _weights(self):
        return [self.model.store.data[0].detach().cpu().clone()]

    def update(self, weights, seed: int):
        raise NotImplementedError


class GradientClient(Client):
    def __init__(self, client_data: Subset) -> None:
        super().__init__(client_data, len(client_data))

    def update(self, weights, seed: int):
        self._load(weights)
        st = self.model.store
        st.zero_grad()
        data = _device_data(True)
        data.set_input_spec(self.model.input_spec)
        idx = torch.as_tensor(np.asarray(self.client_data.indices), dtype=torch.int32,
                              device=device).reshape(1, -1)
        x, y = data.batch(idx)
        self.model.train_step(x, y)
        return [st.grad[0].detach().cpu().clone()]


class WeightClient(Client):
    def __init__(self, client_data: Subset, lr: float, batch_size: int, nr_epochs: int) -> None:
        super().__init__(client_data, batch_size)
        self.lr, self.nr_epochs = lr, nr_epochs
        self.trainer = None

    def update(self, weights, seed: int):
        self._load(weights)
        data = _device_data(True)
        data.set_input_spec(self.model.input_spec)
        if self.trainer is None:
            self.trainer = LocalTrainer(self.model, data, self.lr, self.batch_size, planner="torch",
                                        use_graph=False)
        self.generator.manual_seed(seed)
        self.trainer.run([np.asarray(self.client_data.indices)], [seed], self.nr_epochs,
                         generators=[self.generator])
        return self._weights()


# ------------------------------------------------------------------------------- servers
class Server:
    def __init__(self, lr: float, batch_size: int, seed: int) -> None:
        self.lr, self.batch_size, self.seed = lr, batch_size, seed
        torch.manual_seed(seed)
        self.model = MnistCnn()
        self.clients: list = []

    def test(self) -> float:
        data = _device_data(False)
        data.set_input_spec(self.model.input_spec)
        n = len(data)
        correct = 0
        with torch.no_grad():
            for s in range(0, n, 2000):
                idx = torch.arange(s, min(n, s + 2000), dtype=torch.int32, device=device).reshape(1, -1)
                x, y = data.batch(idx)
                logits, _ = self.model.forward_native(x, False)
                _, _, c = Fn.cross_entropy(logits, y, ncls=10, want_grad=False, with_correct=True)
                correct += int(c.sum().item())
        return 100.0 * correct / n

    def run(self, nr_rounds: int) -> RunResult:
        raise NotImplementedError


class CentralizedServer(Server):
    """Plain mini-batch SGD over the whole training set (reference :193-216)."""

    def __init__(self, lr: float, batch_size: int, seed: int) -> None:
        super().__init__(lr, batch_size, seed)
        self.generator = torch.Generator()
        data = _device_data(True)
        data.set_input_spec(self.model.input_spec)
        self.trainer = LocalTrainer(self.model, data, lr, batch_size, planner="torch")

    def run(self, nr_rounds: int) -> RunResult:
        import time
        res = RunResult("Centralized", 1, 1, self.batch_size, 1, self.lr, self.seed)
        elapsed = 0.0
        all_idx = np.arange(len(_device_data(True)))
        for epoch in range(nr_rounds):
            if device.type == "cuda":
                torch.cuda.synchronize()
            t0 = time.perf_counter()
            self.generator.manual_seed(self.seed + epoch + 1)
            self.trainer.run([all_idx], [self.seed + epoch + 1], 1, generators=[self.generator])
            if device.type == "cuda":
                torch.cuda.synchronize()
            elapsed += time.perf_counter() - t0
            res.wall_time.append(round(elapsed, 1))
            res.message_count.append(0)
            res.test_accuracy.append(self.test())
        return res


class DecentralizedServer(Server):
    """Holds the federated round protocol state; the engines below do the work."""

    def __init__(self, lr: float, batch_size: int, client_subsets: list, client_fraction: float,
                 seed: int) -> None:
        self.lr, self.batch_size, self.seed = lr, batch_size, seed
        self.nr_clients = len(client_subsets)
        self.client_fraction = client_fraction
        self.client_sample_counts = [len(s) for s in client_subsets]
        self.nr_clients_per_round = max(1, round(client_fraction * self.nr_clients))
        self.client_subsets = client_subsets
        self.engine = None

    @property
    def model(self):
        return self.engine.net

    def _make(self, cls, **kw):
        ctx = rdist.context()
        data = _device_data(True)
        test = _device_data(False)
        self.engine = cls(mnist_cnn, data, _indices(self.client_subsets), lr=self.lr,
                          client_fraction=self.client_fraction, seed=self.seed, test_data=test,
                          planner="torch", init_fn=_init_like_reference(self.seed), ctx=ctx, **kw)

    def test(self) -> float:
        return self.engine.test()

    def run(self, nr_rounds: int) -> RunResult:
        return self.engine.run(nr_rounds)


class FedSgdGradientServer(DecentralizedServer):
    def __init__(self, lr: float, client_subsets: list, client_fraction: float, seed: int) -> None:
        super().__init__(lr, -1, client_subsets, client_fraction, seed)
        self._make(FedSGD, name="FedSGDGradient")


class FedAvgServer(DecentralizedServer):
    def __init__(self, lr: float, batch_size: int, client_subsets: list, client_fraction: float,
                 nr_local_epochs: int, seed: int) -> None:
        super().__init__(lr, batch_size, client_subsets, client_fraction, seed)
        self.nr_local_epochs = nr_local_epochs
        self._make(FedAvg, batch_size=batch_size, local_epochs=nr_local_epochs, name="FedAvg")


class FedSgdWeightServer(DecentralizedServer):
    """Homework A1 done right: weights are exchanged, one full-batch local step."""

    def __init__(self, lr: float, client_subsets: list, client_fraction: float, seed: int) -> None:
        super().__init__(lr, -1, client_subsets, client_fraction, seed)
        self._make(FedSgdWeight, name="FedSGDWeight")


__all__ = ["device", "data_path", "ETA", "transform", "train_dataset", "test_loader", "MnistCnn",
           "train_epoch", "split", "RunResult", "Client", "Server", "CentralizedServer",
           "DecentralizedServer", "GradientClient", "WeightClient", "FedSgdGradientServer",
           "FedAvgServer", "FedSgdWeightServer", "configure"]
