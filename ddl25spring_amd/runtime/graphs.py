"""HIP-graph replay of a static training-step callable.

The client-batched FL engine captures whole rounds itself (``fl/local.py``); this is the same
mechanism for torch-style loops over ``nn.Module`` nets (the VFL split-NN, the federated DCGAN,
notebook-style loops): a step of a small net is dozens of launches whose host-side cost (Python,
autograd, launch API) exceeds their GPU time, and one graph launch replaces all of them.

Contract of the callable: every call uses the same tensors (fill static input buffers before the
call) and shapes; anything it computes on the host is frozen at capture, so per-step state must
live on the device (``optim.FlatAdam`` keeps its Adam step counter in ``t_dev`` for this; torch's
own optimizers need ``capturable=True``). Random draws (``torch.randn`` on the device) are
graph-safe: each replay advances the generator's Philox offset.

Each call performs exactly one step: the first ``warmup`` calls run eagerly on a side stream (the
kernels' autotuning and the allocator's first allocations happen there), the next call captures
and then replays once, later calls replay.
"""
from __future__ import annotations

import torch

# Capture mode of every HIP graph the framework records: errors only on unsafe calls of the
# capturing thread. Under "global" (torch's default) an unsafe call on ANY thread fails the
# capture, e.g. a collective library's watchdog thread polling its work events while a
# multi-rank run (bench.py over RCCL) captures its first round.
CAPTURE_MODE = "thread_local"


class CapturedStep:
    def __init__(self, fn, warmup: int = 2, enabled: bool = True):
        self.fn = fn
        self.warmup = warmup
        self.enabled = enabled and torch.cuda.is_available()
        self.calls = 0
        self.graph = None
        self.out = None

    def __call__(self):
        if not self.enabled:
            return self.fn()
        if self.calls < self.warmup:
            self.calls += 1
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                out = self.fn()
            torch.cuda.current_stream().wait_stream(s)
            return out
        if self.graph is None:
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph, capture_error_mode=CAPTURE_MODE):
                self.out = self.fn()
        self.calls += 1
        self.graph.replay()
        return self.out
