"""Per-step scratch arena for small zero-initialised fp32 buffers (BN statistics, BN backward sums
and coefficients, loss accumulators).

A training step needs ~40 such buffers; allocating each with ``torch.zeros`` costs one memset
launch apiece. The arena is zeroed once at the start of the step (a single memset node in the
captured HIP graph) and sliced out sequentially. Its capacity is learned on the first (eager)
step, so graph capture never allocates.
"""
from __future__ import annotations

import math

import torch

_CURRENT: "Workspace | None" = None


class Workspace:
    def __init__(self):
        self.buf: torch.Tensor | None = None
        self.off = 0
        self.need = 0
        self.active = False

    def begin(self, device):
        global _CURRENT
        if self.buf is None or self.buf.numel() < self.need or self.buf.device != torch.device(device):
            if self.need:
                self.buf = torch.empty(self.need, dtype=torch.float32, device=device)
        if self.buf is not None:
            self.buf.zero_()
        self.off = 0
        self.active = True
        _CURRENT = self
        return self

    def end(self):
        global _CURRENT
        self.active = False
        if _CURRENT is self:
            _CURRENT = None

    def take(self, shape, device) -> torch.Tensor:
        n = math.prod(shape)
        n16 = (n + 15) // 16 * 16
        start = self.off
        self.off += n16
        self.need = max(self.need, self.off)
        if self.buf is not None and self.off <= self.buf.numel() and self.buf.device == torch.device(device):
            return self.buf[start:start + n].view(shape)
        return torch.zeros(shape, dtype=torch.float32, device=device)


def zeros(shape, device) -> torch.Tensor:
    """Zeroed fp32 scratch: from the active step arena if there is one, else torch.zeros."""
    ws = _CURRENT
    if ws is not None and ws.active:
        return ws.take(tuple(shape), device)
    return torch.zeros(shape, dtype=torch.float32, device=device)


def scratch(shape, device) -> torch.Tensor:
    """Uninitialised-OK fp32 scratch (same arena; contents are zero but callers must not rely)."""
    return zeros(shape, device)


def scratch_uninit(shape, device) -> torch.Tensor:
    """Scratch that its kernel fully writes before reading: the step arena's slice when one is
    active (graph capture never allocates), else ``torch.empty`` (no memset launch)."""
    ws = _CURRENT
    if ws is not None and ws.active:
        return ws.take(tuple(shape), device)
    return torch.empty(tuple(shape), dtype=torch.float32, device=device)
