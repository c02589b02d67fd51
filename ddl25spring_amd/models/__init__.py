"""Model zoo: native (flat-store, client-batched) nets + torch reference twins."""
from .net import Net  # noqa: F401
from .resnet import resnet18_cifar, resnet18_imagenet, resnet50_imagenet  # noqa: F401
from .zoo import heart_disease_nn, mnist_cnn, mnist_mlp  # noqa: F401
