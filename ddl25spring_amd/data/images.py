"""Image datasets: MNIST / CIFAR-10 / ImageNet *shapes*, device-resident.

There is no network access, so the datasets are synthetic by default — uint8 HWC images with the
real datasets' shapes, sizes and normalisation constants, generated *learnable* (each class has a
fixed random template; samples are template + noise + random shift) so accuracy curves are
meaningful in tests. If a local torchvision MNIST/CIFAR copy exists (``DDL_DATA_ROOT``), it is
used instead (reference hfl_complete.py:7,19-31 downloads MNIST at import time; here nothing is
downloaded and nothing happens at import).

:class:`DeviceImageDataset` keeps the whole uint8 training set in HBM (MNIST 47 MB, CIFAR-10
150 MB) and produces batches with one gather+normalise(+stem-im2col) kernel launch
(``ops.prep_images``) — the MI355X replacement for a per-client ``DataLoader``.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from pathlib import Path

import numpy as np
import torch

from ..ops import functional as Fn

SHAPES = {
    #            H   W   C  classes  n_train  n_test   mean                       std
    "mnist": (28, 28, 1, 10, 60000, 10000, (0.1307,), (0.3081,)),
    "cifar10": (32, 32, 3, 10, 50000, 10000, (0.4914, 0.4822, 0.4465), (0.2470, 0.2435, 0.2616)),
    "imagenet": (224, 224, 3, 1000, 1281167, 50000, (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)),
}


@dataclass
class ImageArrays:
    images: np.ndarray  # uint8 [n, H, W, C]
    labels: np.ndarray  # int64 [n]
    kind: str
    synthetic: bool

    @property
    def targets(self):
        return self.labels

    def __len__(self):
        return len(self.labels)


def synthetic_images(kind: str, n: int, seed: int = 0, learnable: bool = True,
                     num_classes: int | None = None) -> ImageArrays:
    H, W, C, ncls, *_ = SHAPES[kind]
    ncls = num_classes or ncls
    rng = np.random.default_rng(seed)
    labels = rng.integers(0, ncls, n)
    if not learnable:
        imgs = rng.integers(0, 256, (n, H, W, C), dtype=np.uint8)
        return ImageArrays(imgs, labels, kind, True)
    trng = np.random.default_rng(1234 + ncls)  # templates shared by train and test splits
    templ = trng.normal(0, 1, (ncls, H, W, C)).astype(np.float32)
    # smooth the templates a little so conv nets have spatial structure to pick up
    templ = (templ + np.roll(templ, 1, 1) + np.roll(templ, 1, 2)) / 3.0
    imgs = np.empty((n, H, W, C), dtype=np.uint8)
    chunk = 4096
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        base = templ[labels[s:e]]
        # per-sample contrast jitter + pixel noise (no shared shifts: train/test stay aligned)
        gain = rng.uniform(0.7, 1.3, (e - s, 1, 1, 1))
        x = 128 + 48 * gain * base + rng.normal(0, 36, base.shape)
        imgs[s:e] = np.clip(x, 0, 255).astype(np.uint8)
    return ImageArrays(imgs, labels, kind, True)


def _try_torchvision(kind: str, train: bool):
    root = os.environ.get("DDL_DATA_ROOT")
    if not root:
        return None
    try:
        from torchvision import datasets  # noqa: F401
    except Exception:
        return None
    try:
        if kind == "mnist":
            ds = datasets.MNIST(root, train=train, download=False)
            imgs = ds.data.numpy()[..., None]
            return ImageArrays(imgs.astype(np.uint8), ds.targets.numpy(), kind, False)
        if kind == "cifar10":
            ds = datasets.CIFAR10(root, train=train, download=False)
            return ImageArrays(ds.data.astype(np.uint8), np.array(ds.targets), kind, False)
    except Exception:
        return None
    return None


def load_images(kind: str, train: bool = True, n: int | None = None, seed: int = 0) -> ImageArrays:
    """Real dataset if a local copy exists (DDL_DATA_ROOT), else the synthetic stand-in."""
    real = _try_torchvision(kind, train)
    if real is not None:
        if n is not None:
            real = ImageArrays(real.images[:n], real.labels[:n], kind, False)
        return real
    _, _, _, _, ntr, nte, *_ = SHAPES[kind]
    n = n if n is not None else (ntr if train else nte)
    return synthetic_images(kind, n, seed=seed + (0 if train else 99991))


class DeviceImageDataset:
    """Whole uint8 dataset in device memory + batch materialisation for a given model input spec."""

    def __init__(self, arrays: ImageArrays, device, input_spec: dict | None = None):
        self.kind = arrays.kind
        H, W, C, ncls, _, _, mean, std = SHAPES[arrays.kind]
        self.num_classes = ncls
        self.device = torch.device(device)
        self.images = torch.from_numpy(np.ascontiguousarray(arrays.images)).to(self.device)
        self.labels = torch.from_numpy(arrays.labels.astype(np.int32)).to(self.device)
        self.mean = torch.tensor(mean, dtype=torch.float32, device=self.device)
        self.inv_std = 1.0 / torch.tensor(std, dtype=torch.float32, device=self.device)
        self.synthetic = arrays.synthetic
        self.set_input_spec(input_spec or {})

    def set_input_spec(self, spec: dict):
        self.spec = dict(spec)
        self.dtype = torch.float32 if spec.get("dtype") == "fp32" else torch.bfloat16
        self.cpad = spec.get("cpad", 32)
        self.k = spec.get("stem_k", 0) if spec.get("im2col") else 0
        self.pad = spec.get("pad", 0)
        self.stride = spec.get("stem_stride", 1)
        self.flat = spec.get("flat", False)

    def __len__(self):
        return self.labels.numel()

    def batch(self, idx: torch.Tensor, out: torch.Tensor | None = None):
        """idx int32 [G, B] (device) -> (x [G, B, H', W', cpad] | [G, B, F] in the spec's activation
        dtype (bf16 / fp32), y int32 [G, B]). One launch gathers images and labels."""
        G, B = idx.shape
        y = torch.empty(G, B, dtype=torch.int32, device=self.device)
        kw = dict(labels=self.labels, labels_out=y)
        if self.flat:
            x = Fn.prep_images(self.images, idx, self.mean, self.inv_std, 8, 0, 0, 1, dtype=self.dtype, **kw)
            # [n, H, W, 8] -> keep the real channel(s), flatten, pad to cpad
            C = self.images.shape[-1]
            flat = x[..., :C].reshape(G, B, -1)
            xo = torch.zeros(G, B, self.cpad, dtype=self.dtype, device=self.device)
            xo[..., :flat.shape[-1]] = flat
        else:
            x = Fn.prep_images(self.images, idx, self.mean, self.inv_std, self.cpad,
                               self.k, self.pad, self.stride, out=out, dtype=self.dtype, **kw)
            xo = x.reshape(G, B, *x.shape[1:])
        return xo, y

    def full(self, n: int | None = None):
        n = n or len(self)
        idx = torch.arange(n, dtype=torch.int32, device=self.device).reshape(1, n)
        return self.batch(idx)
