"""Tracing / metrics: device-event phase timers, roctx ranges, JSONL logs.

The reference times phases with ``time.perf_counter`` around host code (hfl_complete.py:274-307);
on an asynchronous GPU that measures launch, not execution. Here:

* ``PhaseTimer``  — per-phase GPU time from HIP events recorded on the current stream (no
  synchronisation inside the loop; ``summary()`` syncs once), host perf_counter on CPU.
* ``range(name)`` — roctx push/pop (``libroctx64``) so phases appear as named regions in
  ``rocprofv3 --marker-trace`` / rocpd timelines; a no-op if the library is absent.
* ``JsonlLogger`` — one JSON object per line (round metrics, throughput), rank-0 only by default.
"""
from __future__ import annotations

import contextlib
import ctypes
import json
import os
import time
from collections import defaultdict

import torch

_roctx = None


def _roctx_lib():
    global _roctx
    if _roctx is None:
        _roctx = False
        for name in ("libroctx64.so", "/opt/rocm/lib/libroctx64.so"):
            try:
                lib = ctypes.CDLL(name)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                lib.roctxRangePushA.restype = ctypes.c_int
                lib.roctxRangePop.restype = ctypes.c_int
                _roctx = lib
                break
            except OSError:
                continue
    return _roctx or None


@contextlib.contextmanager
def range(name: str):  # noqa: A001 - mirrors roctx naming
    lib = _roctx_lib()
    if lib is not None:
        lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        if lib is not None:
            lib.roctxRangePop()


class PhaseTimer:
    """timer = PhaseTimer(device); with timer("local_train"): ...; timer.summary() -> {phase: ms}"""

    def __init__(self, device=None, markers: bool = True):
        self.device = torch.device(device) if device is not None else None
        self.gpu = self.device is not None and self.device.type == "cuda"
        self.markers = markers
        self._events = defaultdict(list)  # phase -> [(start, end)]
        self._host = defaultdict(float)

    @contextlib.contextmanager
    def __call__(self, phase: str):
        ctx = range(phase) if self.markers else contextlib.nullcontext()
        with ctx:
            if self.gpu:
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                try:
                    yield
                finally:
                    e.record()
                    self._events[phase].append((s, e))
            else:
                t0 = time.perf_counter()
                try:
                    yield
                finally:
                    self._host[phase] += (time.perf_counter() - t0) * 1e3

    def summary(self, reset: bool = True) -> dict:
        out = dict(self._host)
        if self._events:
            torch.cuda.synchronize(self.device)
            for ph, evs in self._events.items():
                out[ph] = out.get(ph, 0.0) + sum(s.elapsed_time(e) for s, e in evs)
        if reset:
            self._events.clear()
            self._host.clear()
        return {k: round(v, 3) for k, v in out.items()}


class JsonlLogger:
    def __init__(self, path: str | None, rank: int = 0, all_ranks: bool = False):
        self.enabled = path is not None and (all_ranks or rank == 0)
        self.rank = rank
        self.f = None
        if self.enabled:
            os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
            self.f = open(path, "a", buffering=1)

    def log(self, **rec):
        if self.f is not None:
            rec.setdefault("time", time.time())
            rec.setdefault("rank", self.rank)
            self.f.write(json.dumps(rec, default=float) + "\n")

    def close(self):
        if self.f is not None:
            self.f.close()
            self.f = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def read_jsonl(path: str) -> list[dict]:
    with open(path) as f:
        return [json.loads(line) for line in f if line.strip()]
