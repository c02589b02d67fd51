"""Pipeline schedule IR (built and verified by the native runtime, csrc/runtime/runtime.cpp).

Ops per stage: FWD / BWD of a micro-batch, SEND/RECV of activations (downstream) and gradients
(upstream). Consecutive comm ops with the same ``group`` id are posted together (one
``batch_isend_irecv``), which is how 1F1B's "send activation + receive gradient" exchange avoids the
ordering deadlock of the reference's attempt (intro_PP_1F1B_MP.py:86-157; out_MP*.txt hang).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from ..ops import _lib

FWD, BWD, SEND_ACT, RECV_ACT, SEND_GRAD, RECV_GRAD = range(6)
OP_NAMES = ["FWD", "BWD", "SEND_ACT", "RECV_ACT", "SEND_GRAD", "RECV_GRAD"]
KINDS = {"naive": 0, "gpipe": 1, "1f1b": 2}


@dataclass(frozen=True)
class Action:
    stage: int
    op: int
    mb: int
    peer: int
    group: int

    def __repr__(self):
        p = f"->{self.peer}" if self.op in (SEND_ACT, SEND_GRAD) else (f"<-{self.peer}" if self.op in (RECV_ACT, RECV_GRAD) else "")
        g = f" g{self.group}" if self.group >= 0 else ""
        return f"{OP_NAMES[self.op]}({self.mb}){p}{g}"


def _as_array(actions) -> np.ndarray:
    return np.ascontiguousarray(np.array([[a.stage, a.op, a.mb, a.peer, a.group] for a in actions],
                                         dtype=np.int32).reshape(-1, 5))


def build(kind: str, n_stages: int, n_micro: int) -> list[Action]:
    lib = _lib.runtime()
    cap = 16 * n_stages * n_micro + 64
    buf = np.zeros((cap, 5), dtype=np.int32)
    n = lib.ddl_sched_build(KINDS[kind], n_stages, n_micro,
                            buf.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), cap)
    if n < 0:
        raise RuntimeError("schedule buffer too small")
    return [Action(*map(int, row)) for row in buf[:n]]


def verify(actions: list[Action], n_stages: int) -> int:
    """0 = deadlock-free and FIFO-consistent; >0 = 1+index of a blocked action; <0 = mismatch."""
    arr = _as_array(actions)
    return int(_lib.runtime().ddl_sched_verify(arr.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                               len(actions), n_stages))


def stage_program(actions: list[Action], stage: int) -> list[list[Action]]:
    """The stage's actions as a list of steps; a step is one compute op or one posted comm group."""
    prog = [a for a in actions if a.stage == stage]
    steps, i = [], 0
    while i < len(prog):
        a = prog[i]
        if a.op in (FWD, BWD) or a.group < 0:
            steps.append([a])
            i += 1
        else:
            j = i
            while j < len(prog) and prog[j].group == a.group and prog[j].op not in (FWD, BWD):
                j += 1
            steps.append(prog[i:j])
            i = j
    return steps


def make(kind: str, n_stages: int, n_micro: int) -> list[Action]:
    acts = build(kind, n_stages, n_micro)
    rc = verify(acts, n_stages)
    if rc != 0:
        raise RuntimeError(f"{kind} schedule S={n_stages} M={n_micro} failed verification ({rc})")
    return acts
