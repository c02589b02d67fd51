"""Client data partitioning (horizontal FL) and mini-batch planning.

``split`` reproduces reference hfl_complete.py:91-104 bit-for-bit (same numpy ``default_rng``
calls): IID = ``array_split(rng.permutation(n), N)``; non-IID = McMahan's pathological split
(sort by label, 2N shards, each client gets 2 random shards). Labels come from the dataset's
``targets`` array instead of iterating the transformed dataset.

``plan_epoch`` is the per-round batch table for the device loader (native C++ planner in
csrc/runtime/runtime.cpp, or torch.randperm for DataLoader-identical shuffles).
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from ..ops import _lib


def split(nr_clients: int, iid: bool, seed: int, labels=None, n: int | None = None) -> list[np.ndarray]:
    """-> list of int64 index arrays, one per client (same RNG call sequence as the reference)."""
    rng = np.random.default_rng(seed)
    if labels is not None:
        labels = np.asarray(labels)
        n = len(labels)
    if iid:
        return [np.asarray(s, dtype=np.int64) for s in np.array_split(rng.permutation(n), nr_clients)]
    if labels is None:
        raise ValueError("non-IID split needs labels")
    sorted_idx = np.argsort(labels)
    shards = np.array_split(sorted_idx, 2 * nr_clients)
    order = rng.permutation(len(shards))
    return [np.concatenate([shards[i] for i in pair], dtype=np.int64)
            for pair in order.reshape(nr_clients, 2)]


def mix_seed(*parts: int) -> int:
    h = 0x243F6A8885A308D3
    for p in parts:
        h ^= (int(p) + 0x9E3779B97F4A7C15 + ((h << 6) & 0xFFFFFFFFFFFFFFFF) + (h >> 2))
        h &= 0xFFFFFFFFFFFFFFFF
    return h


def plan_epoch(client_indices: list[np.ndarray], batch: int, seeds: list[int], shuffle: bool = True,
               planner: str = "native") -> np.ndarray:
    """-> int32 [steps, G, batch]; entries past a client's end are -1. All clients equal size."""
    G = len(client_indices)
    count = len(client_indices[0])
    assert all(len(c) == count for c in client_indices), "clients in one plan must be equal-size"
    steps = (count + batch - 1) // batch
    if planner == "torch":
        out = -np.ones((steps, G, batch), dtype=np.int32)
        for g, (ci, sd) in enumerate(zip(client_indices, seeds)):
            gen = torch.Generator().manual_seed(int(sd) & 0x7FFFFFFFFFFFFFFF)
            # first epoch of DataLoader(shuffle=True, generator=gen): the loader's base-seed draw
            # precedes the sampler's randperm (see fl.local.LocalTrainer._torch_plan)
            torch.empty((), dtype=torch.int64).random_(generator=gen)
            perm = torch.randperm(count, generator=gen).numpy() if shuffle else np.arange(count)
            seq = np.asarray(ci)[perm]
            for s in range(steps):
                chunk = seq[s * batch:(s + 1) * batch]
                out[s, g, :len(chunk)] = chunk
        return out
    lib = _lib.runtime()
    idx = np.ascontiguousarray(np.stack(client_indices).astype(np.int32))
    sd = np.ascontiguousarray(np.asarray([s & 0xFFFFFFFFFFFFFFFF for s in seeds], dtype=np.uint64))
    out = np.empty((steps, G, batch), dtype=np.int32)
    got = lib.ddl_plan_epoch(idx.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), G, count, batch,
                             sd.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), int(shuffle),
                             out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
    assert got == steps
    return out
