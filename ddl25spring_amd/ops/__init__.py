"""Op layer: HIP/CDNA4 kernels (device) + PyTorch reference (CPU) behind one functional API."""
from . import functional  # noqa: F401
from .functional import ConvGeom  # noqa: F401
