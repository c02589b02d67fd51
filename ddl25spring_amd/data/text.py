"""Token stream stand-ins for simplellm's ``SPTokenizer`` and ``TinyStories``.

The reference streams TinyStories through a SentencePiece tokenizer (~32k vocab, inferred from
the first-iteration loss 10.57 ~ ln 32000). Neither the dataset nor the tokenizer model
is available offline, so:
  * ``SPTokenizer`` keeps the interface (``vocab_size``, ``pad_id``, ``encode``/``decode``) with a
    deterministic byte-level scheme (ids 3..258 = bytes, 0 pad, 1 bos, 2 eos) inside a 32000-id
    vocabulary (the unused ids keep the embedding / LM-head shapes of the reference);
  * ``TinyStories(tokenizer, batch_size, seq_l, skip)`` yields ``[batch_size, seq_l]`` int64
    batches from a fixed synthetic "story grammar" (a sparse random bigram Markov chain over a
    2,048-token sub-vocabulary), so next-token loss genuinely decreases. ``skip`` offsets the
    stream exactly like the reference's per-rank / per-pipeline ``skip=rank*5000``.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from ..ops import _lib


class SPTokenizer:
    def __init__(self, vocab_size: int = 32000):
        self.vocab_size = vocab_size
        self.pad_id, self.bos_id, self.eos_id = 0, 1, 2

    def encode(self, text: str) -> list[int]:
        return [self.bos_id] + [3 + b for b in text.encode("utf-8")]

    def decode(self, ids) -> str:
        return bytes(int(i) - 3 for i in ids if 3 <= int(i) < 259).decode("utf-8", "replace")


class TinyStories:
    def __init__(self, tokenizer: SPTokenizer, batch_size: int = 3, seq_l: int = 256, skip: int = 0,
                 seed: int = 1234, sub_vocab: int = 2048, branching: int = 8):
        self.tok, self.B, self.S = tokenizer, batch_size, seq_l
        self.skip = skip
        rng = np.random.default_rng(seed)
        V = min(sub_vocab, tokenizer.vocab_size - 3)
        self.V = V
        self.next_tok = rng.integers(3, 3 + V, (V + 3, branching))
        p = rng.dirichlet(np.full(branching, 0.3), V + 3)
        self.cum = np.cumsum(p, 1)
        self.seed = seed
        self._next = np.ascontiguousarray(self.next_tok, dtype=np.int64)
        self._cum = np.ascontiguousarray(self.cum, dtype=np.float64)

    def _sequence(self, index: int) -> np.ndarray:
        rng = np.random.default_rng((self.seed, index))
        out = np.empty(self.S, dtype=np.int64)
        out[0] = self.tok.bos_id
        cur = int(rng.integers(3, 3 + self.V))
        u = rng.random(self.S)
        for t in range(1, self.S):
            out[t] = cur
            j = int(np.searchsorted(self.cum[cur], u[t]))
            cur = int(self.next_tok[cur, min(j, self.next_tok.shape[1] - 1)])
        return out

    def batch(self, start: int) -> np.ndarray:
        """Sequences start .. start+B-1, identical to ``_sequence``: numpy draws each sequence's
        first token and uniforms from (seed, index); the chain walk runs in the C++ runtime
        (``ddl_markov_walk``) — the per-token Python loop cost ~25 ms per 32x256 batch, longer
        than the GPU step it feeds."""
        B, S = self.B, self.S
        cur0 = np.empty(B, dtype=np.int64)
        U = np.empty((B, S), dtype=np.float64)
        for b in range(B):
            rng = np.random.default_rng((self.seed, start + b))
            cur0[b] = rng.integers(3, 3 + self.V)
            U[b] = rng.random(S)
        out = np.empty((B, S), dtype=np.int64)
        i64p, f64p = ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_double)
        _lib.runtime().ddl_markov_walk(self._next.ctypes.data_as(i64p), self._cum.ctypes.data_as(f64p),
                                       self._next.shape[1], cur0.ctypes.data_as(i64p),
                                       U.ctypes.data_as(f64p), B, S, self.tok.bos_id,
                                       out.ctypes.data_as(i64p))
        return out

    def __iter__(self):
        i = self.skip * self.B
        while True:
            yield torch.from_numpy(self.batch(i))
            i += self.B
