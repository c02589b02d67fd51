"""Model zoo on the native layer library.

* :func:`mnist_cnn` — MnistCnn of reference hfl_complete.py:39-64 (conv 1->32->64, max-pool,
  dropout .25/.5, fc 9216->128->10, log-softmax output), 1,199,882 params.
* :func:`mnist_mlp` — "FedAvg 2-client MLP on MNIST-shaped tensors" (BASELINE config 1).
* :func:`heart_disease_nn` — HeartDiseaseNN of reference lab/tutorial_2a/centralized.py:13-28.
* ResNet-18 / ResNet-50 live in :mod:`.resnet`.
"""
from __future__ import annotations

import torch

from . import convert
from .layers import ConvUnit, Dropout, Flatten, Linear, MaxPool2
from .net import Net


class LogSoftmaxNet(Net):
    """Net whose torch-facing output is log_softmax(logits) (MnistCnn's F.log_softmax)."""

    def output_transform(self, logits):
        return torch.log_softmax(logits, -1)

    def output_transform_backward(self, out, grad):
        # d/dz of log_softmax: g - softmax * sum(g)
        return grad - torch.exp(out) * grad.sum(-1, keepdim=True)


def mnist_cnn(groups: int = 1, precision: str | None = None) -> Net:
    conv1 = ConvUnit(32, 32, k=1, stride=1, pad=0, bias=True, act="relu", cin_true=9, fan_in=9)
    conv1.pname = "conv1"
    conv2 = ConvUnit(32, 64, k=3, stride=1, pad=0, bias=True, act="relu")
    conv2.pname = "conv2"
    fc1 = Linear(9216, 128, bias=True, act="relu")
    fc1.pname = "fc1"
    fc2 = Linear(128, 10, bias=True)
    fc2.pname = "fc2"
    layers = [conv1, conv2, MaxPool2(), Dropout(0.25), Flatten(), fc1, Dropout(0.5), fc2]
    return LogSoftmaxNet(layers, groups=groups, num_classes=10,
                         input_spec={"cpad": 32, "im2col": True, "stem_k": 3, "pad": 0},
                         name="mnist_cnn", precision=precision)


def mnist_cnn_mapping():
    return [("conv1.weight", "conv1.weight", "stem", None), ("conv1.bias", "conv1.bias", "vec", None),
            ("conv2.weight", "conv2.weight", "conv", None), ("conv2.bias", "conv2.bias", "vec", None),
            ("fc1.weight", "fc1.weight", "linear", (64, 12, 12)), ("fc1.bias", "fc1.bias", "vec", None),
            ("fc2.weight", "fc2.weight", "linear", None), ("fc2.bias", "fc2.bias", "vec", None)]


def mnist_mlp(groups: int = 1, hidden=(200, 200), num_classes: int = 10, precision: str | None = None) -> Net:
    dims = (784, *hidden, num_classes)
    layers = []
    for i, (a, b) in enumerate(zip(dims[:-1], dims[1:])):
        last = i == len(dims) - 2
        fin = 800 if i == 0 else a  # 784 padded to a multiple of 32
        lin = Linear(fin, b, bias=True, act=None if last else "relu", fin_true=a, fan_in=a)
        lin.pname = f"layers.{i}"
        layers.append(lin)
    return Net(layers, groups=groups, num_classes=num_classes, input_spec={"cpad": 800, "flat": True},
               name="mnist_mlp", precision=precision)


def mnist_mlp_mapping(n_layers=3):
    m = []
    for i in range(n_layers):
        m.append((f"layers.{i}.weight", f"layers.{i}.weight", "linear", None))
        m.append((f"layers.{i}.bias", f"layers.{i}.bias", "vec", None))
    return m


def heart_disease_nn(groups: int = 1, in_features: int = 30, precision: str | None = None) -> Net:
    """30 -> 64 -> 128 -> 256 -> 2, LeakyReLU, Dropout(0.1) before the last layer."""
    l1 = Linear(in_features, 64, act="leaky_relu")
    l1.pname = "fc1"
    l2 = Linear(64, 128, act="leaky_relu")
    l2.pname = "fc2"
    l3 = Linear(128, 256, act="leaky_relu")
    l3.pname = "fc3"
    l4 = Linear(256, 2)
    l4.pname = "fc4"
    return Net([l1, l2, l3, Dropout(0.1), l4], groups=groups, num_classes=2, name="heart_disease_nn",
               precision=precision)


def import_mnist_cnn(net: Net, module) -> None:
    convert.import_torch(net, module, mnist_cnn_mapping())
