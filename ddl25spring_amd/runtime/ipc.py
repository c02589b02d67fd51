"""All-reduce by direct peer reads over xGMI (hipIPC-mapped uncached buffers).

The small-message path of the communication layer. RCCL's ring is
latency-bound for the messages the labs exchange (the FedAvg / FedSGD weighted reduce of a
4.8 MB MnistCnn, reference hfl_complete.py:370-378; KB-sized VFL and pipeline tensors): each GPU
here instead reads its peers' buffers directly, over all of its xGMI links at once, in one kernel
launch (``csrc/kernels/ipc_allreduce.hip``):

* one-shot (n*4 < ``two_shot_bytes``): every rank sums the whole vector from every peer;
* two-shot: reduce-scatter by peer reads into a result slot, then all-gather by peer reads.

Both sum in rank order, so every rank gets bit-identical results (replicated FL server state
stays identical without a broadcast). Setup is collective: every rank allocates one uncached
buffer, the IPC handles are exchanged over the process group, every rank maps every peer's.

``IpcAllReduce.all_reduce(t)`` takes an fp32 contiguous device tensor of at most ``capacity``
bytes and reduces it in place (SUM). A barrier wait that exceeds ``timeout_s`` (a peer that never
arrives) sets an error word instead of hanging the GPU; ``check()`` raises on it.

The path is used by :class:`ddl25spring_amd.runtime.dist.DistContext` by default
(``DDL_IPC_ALLREDUCE=auto``): at init every rank times it against RCCL at a ladder of sizes and the
peer-read kernel keeps the messages below the measured crossover (``dist.probe_ipc_threshold``);
``DDL_IPC_ALLREDUCE=1`` forces it up to ``DDL_IPC_MAX_BYTES``, ``0`` turns it off.
"""
from __future__ import annotations

import ctypes

import torch
import torch.distributed as dist

from ..ops import _lib
from ..ops._lib import check

IPC_MAXR = 8
_vp, _i32, _i64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong


class IpcArgs(ctypes.Structure):
    _fields_ = [("base", _vp * IPC_MAXR), ("in_", _vp), ("out", _vp), ("n", _i64), ("cap", _i64),
                ("err", _vp), ("timeout", _i64), ("rank", _i32), ("world", _i32),
                ("two_shot", _i32)]


_SIGS = {
    "ddl_ipc_malloc": [_i64, ctypes.POINTER(_vp)],
    "ddl_ipc_free": [_vp],
    "ddl_ipc_get_handle": [_vp, ctypes.c_char_p],
    "ddl_ipc_open": [ctypes.c_char_p, ctypes.POINTER(_vp)],
    "ddl_ipc_close": [_vp],
    "ddl_ipc_allreduce": [ctypes.POINTER(IpcArgs), _i32, _vp],
}


def _lib_ipc():
    _lib.register_signatures(_SIGS)
    lib = _lib.kernels()
    for f in ("ddl_ipc_args_size", "ddl_ipc_handle_size", "ddl_ipc_max_blocks"):
        getattr(lib, f).restype = ctypes.c_int
    if lib.ddl_ipc_args_size() != ctypes.sizeof(IpcArgs):
        raise RuntimeError(f"ABI mismatch for IpcArgs: C {lib.ddl_ipc_args_size()} vs ctypes "
                           f"{ctypes.sizeof(IpcArgs)}")
    return lib


class IpcAllReduce:
    def __init__(self, rank: int, world: int, device, capacity: int = 16 << 20, group=None,
                 two_shot_bytes: int = 512 << 10, nblocks: int = 32, timeout_s: float = 20.0):
        if not 1 <= world <= IPC_MAXR:
            raise ValueError(f"IPC all-reduce supports 1..{IPC_MAXR} ranks (one node), got {world}")
        self.lib = _lib_ipc()
        self.rank, self.world, self.device = rank, world, torch.device(device)
        self.cap = (int(capacity) + 15) // 16 * 16
        self.two_shot_bytes = two_shot_bytes
        self.nblocks = max(1, min(nblocks, self.lib.ddl_ipc_max_blocks()))
        self.timeout_ticks = int(timeout_s * 1e8)  # s_memrealtime: 100 MHz
        # Setup is failure-agreeing: a rank whose allocation, export or peer mapping fails still
        # takes part in every collective below, and all ranks agree (MAX of a failure flag) before
        # anyone uses the buffers, so either every rank holds the peer-read path or none does
        # (a one-sided failure would otherwise leave ranks on different all-reduce paths).
        self._mine = None
        self.bases: list[_vp] = []
        self._opened: list[_vp] = []
        err = None
        with torch.cuda.device(self.device):
            hsz = self.lib.ddl_ipc_handle_size()
            handle = None
            try:
                mine = _vp()
                check(self.lib.ddl_ipc_malloc(self.cap, ctypes.byref(mine)), "ipc_malloc")
                self._mine = mine
                buf = ctypes.create_string_buffer(64)
                check(self.lib.ddl_ipc_get_handle(mine, buf), "ipc_get_handle")
                handle = buf.raw[:hsz]
            except Exception as e:  # noqa: BLE001 - reported through the agreement below
                err = e
            handles = [handle] * world
            if world > 1:
                dist.all_gather_object(handles, handle, group=group)
            if err is None and any(h is None for h in handles):
                err = RuntimeError("a peer failed to export its IPC buffer")
            if err is None:
                try:
                    for r in range(world):
                        if r == rank:
                            self.bases.append(self._mine)
                            continue
                        p = _vp()
                        check(self.lib.ddl_ipc_open(ctypes.create_string_buffer(handles[r], 64), ctypes.byref(p)),
                              f"ipc_open(rank {r})")
                        self.bases.append(p)
                        self._opened.append(p)
                except Exception as e:  # noqa: BLE001
                    err = e
            self.err = torch.zeros(1, dtype=torch.int32, device=self.device)
            if world > 1:
                fdev = "cpu" if dist.get_backend(group) == "gloo" else self.device
                flag = torch.tensor([0 if err is None else 1], dtype=torch.int32, device=fdev)
                dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=group)
                if err is None and int(flag.item()):
                    err = RuntimeError("a peer failed to map the IPC buffers")
        if err is not None:
            self._release()
            raise RuntimeError(f"ipc all-reduce setup failed on some rank: {err}") from err
        if world > 1:
            dist.barrier(group=group)  # every peer has mapped every buffer before first use
        self.calls = 0

    def all_reduce(self, t: torch.Tensor) -> torch.Tensor:
        """In-place SUM over the ranks of an fp32 contiguous device tensor (<= capacity bytes)."""
        if t.dtype != torch.float32 or not t.is_contiguous() or t.device != self.device:
            raise ValueError("ipc all_reduce: fp32 contiguous tensor on this rank's device")
        if t.numel() * 4 > self.cap:
            raise ValueError(f"ipc all_reduce: {t.numel() * 4} B exceeds the {self.cap} B slot")
        if t.data_ptr() % 16:
            raise ValueError("ipc all_reduce: 16-byte aligned tensor required")
        a = IpcArgs()
        for r, b in enumerate(self.bases):
            a.base[r] = b.value
        a.in_ = a.out = t.data_ptr()
        a.n, a.cap = t.numel(), self.cap
        a.err, a.timeout = self.err.data_ptr(), self.timeout_ticks
        a.rank, a.world = self.rank, self.world
        a.two_shot = int(self.world > 2 and t.numel() * 4 >= self.two_shot_bytes)
        check(self.lib.ddl_ipc_allreduce(ctypes.byref(a), self.nblocks,
                                         torch.cuda.current_stream(self.device).cuda_stream),
              "ipc_allreduce")
        self.calls += 1
        return t

    def all_reduce_ordered(self, t: torch.Tensor) -> torch.Tensor:
        """In-place rank-ORDER sum of an fp32 contiguous device tensor of any size: slot-sized
        chunks, each one peer-read kernel (one- or two-shot, both add the ranks' values in rank
        order: p0 + p1 + ... bitwise on every rank). What the ordered FedAvg mean needs
        (fl/aggregate.py) without all-gathering W full copies."""
        step = self.cap // 4
        flat = t.view(-1)
        for off in range(0, flat.numel(), step):
            self.all_reduce(flat[off:off + step])
        return t

    def check(self):
        """Raise if any barrier of the calls so far timed out (synchronises the device)."""
        if int(self.err.item()):
            raise RuntimeError("ipc all_reduce: a peer did not arrive within the barrier timeout")

    def close(self, group=None):
        """Collective: every rank's last kernel may still be reading MY buffer, so unmap and free only
        after all ranks have drained their device (synchronize + barrier)."""
        torch.cuda.synchronize(self.device)
        if self.world > 1 and dist.is_initialized():
            dist.barrier(group=group)
        self._release()

    def _release(self):
        for p in self._opened:
            self.lib.ddl_ipc_close(p)
        self._opened = []
        if self._mine is not None:
            self.lib.ddl_ipc_free(self._mine)
            self._mine = None
