"""Process / device / communicator bootstrap.

One process per GPU; ``torch.distributed`` with backend ``nccl`` (= RCCL on ROCm, over xGMI) for
device tensors, ``gloo`` for CPU runs and tests. Rendezvous follows the torchrun / reference env
contract (``MASTER_ADDR``/``MASTER_PORT``/``RANK``/``WORLD_SIZE``; reference
lab/tutorial_1b/DP/gradient_aggr/intro_DP_GA.py:11-15 reads the rank from argv and hard-codes
localhost:29500 — both spellings are accepted here).

Sub-communicators are created *collectively* (every rank calls ``new_group`` for every group in
the same order) which fixes the reference's non-collective group creation
(intro_PP_1F1B_MP.py:31-36).
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass, field

import torch
import torch.distributed as dist


@dataclass
class DistContext:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    device: torch.device = field(default_factory=lambda: torch.device("cpu"))
    backend: str = "none"
    groups: dict = field(default_factory=dict)
    ipc: object = None          # runtime.ipc.IpcAllReduce (peer-read all-reduce) when enabled
    ipc_max_bytes: int = 0      # SUM all-reduces of fp32 tensors up to this size take the peer-read path
    ipc_policy: dict = field(default_factory=dict)  # how ipc_max_bytes was chosen (probe table)

    @property
    def is_distributed(self) -> bool:
        return (self.world > 1 or self.forced_pg) and dist.is_initialized()

    @property
    def is_main(self) -> bool:
        return self.rank == 0

    # ------------------------------------------------------------- collectives (no-ops at world 1)
    forced_pg: bool = False     # a process group even at world 1 (RCCL code-path rehearsal)

    def all_reduce(self, t: torch.Tensor, op=None, group=None):
        if self.is_distributed:
            if (self.ipc is not None and group is None and op in (None, dist.ReduceOp.SUM)
                    and t.dtype == torch.float32 and t.is_contiguous() and t.is_cuda
                    and t.numel() * 4 <= self.ipc_max_bytes and t.data_ptr() % 16 == 0):
                self.ipc.all_reduce(t)  # small message: one peer-read kernel over xGMI
            else:
                dist.all_reduce(t, op=op or dist.ReduceOp.SUM, group=group)
        return t

    def broadcast(self, t: torch.Tensor, src: int = 0, group=None):
        if self.is_distributed:
            dist.broadcast(t, src, group=group)
        return t

    def all_gather_into(self, out: torch.Tensor, t: torch.Tensor, group=None):
        if self.is_distributed:
            dist.all_gather_into_tensor(out, t, group=group)
        else:
            out.copy_(t.reshape(out.shape))
        return out

    def all_gather_rows(self, t: torch.Tensor, group=None) -> torch.Tensor:
        """[W, *t.shape]: every rank's t, in rank order (RCCL all-gather into one buffer; gloo via
        its list form)."""
        W = dist.get_world_size(group) if self.is_distributed else 1
        out = torch.empty((W,) + tuple(t.shape), dtype=t.dtype, device=t.device)
        if not self.is_distributed:
            out[0].copy_(t)
        elif self.backend == "nccl":
            dist.all_gather_into_tensor(out, t.contiguous(), group=group)
        else:
            dist.all_gather(list(out.unbind(0)), t.contiguous(), group=group)
        return out

    def all_to_all_single(self, out: torch.Tensor, t: torch.Tensor, group=None):
        if self.is_distributed:
            dist.all_to_all_single(out, t, group=group)
        else:
            out.copy_(t)
        return out

    def check_comm(self):
        """Surface a peer-read all-reduce barrier timeout (sticky device error word) as an exception;
        called at round / sync boundaries (it synchronises the device)."""
        if self.ipc is not None:
            self.ipc.check()

    def barrier(self):
        if self.is_distributed:
            if self.backend == "nccl":
                dist.barrier(device_ids=[self.device.index])
            else:
                dist.barrier()

    def max_scalar(self, v: float) -> float:
        if not self.is_distributed:
            return v
        t = torch.tensor([v], dtype=torch.float64,
                         device=self.device if self.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def sum_scalar(self, v: float) -> float:
        if not self.is_distributed:
            return v
        t = torch.tensor([v], dtype=torch.float64,
                         device=self.device if self.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return float(t.item())

    def new_groups(self, name: str, partition: list[list[int]]):
        """Collective creation of a partition of the ranks into sub-groups; returns my group."""
        mine = None
        for ranks in partition:
            g = dist.new_group(ranks=ranks) if self.is_distributed else None
            if self.rank in ranks:
                mine = g
        self.groups[name] = mine
        return mine


_CTX: DistContext | None = None


def init(backend: str | None = None, device: str | None = None, rank: int | None = None,
         world_size: int | None = None, timeout_s: int = 600) -> DistContext:
    """Initialise from env (torchrun) or explicit args. Safe to call once per process."""
    global _CTX
    if _CTX is not None:
        return _CTX
    rank = int(os.environ.get("RANK", rank if rank is not None else 0))
    world = int(os.environ.get("WORLD_SIZE", world_size if world_size is not None else 1))
    local = int(os.environ.get("LOCAL_RANK", rank))
    want_gpu = device != "cpu" and (device is not None and device.startswith("cuda") or
                                    (device is None and torch.cuda.is_available()))
    # DDL_FORCE_PG=1: create the process group even at world 1, so the collective code paths
    # (init_process_group(device_id=), barrier(device_ids=), device scalars, bucket hooks) run
    forced = os.environ.get("DDL_FORCE_PG", "0") == "1" and world == 1
    if want_gpu:
        ndev = torch.cuda.device_count()
        dev = torch.device("cuda", local % max(ndev, 1))
        torch.cuda.set_device(dev)
    else:
        dev = torch.device("cpu")
        if world > 1 and "OMP_NUM_THREADS" not in os.environ:
            # ranks sharing a host must split its cores, or their intra-op pools oversubscribe it
            local_world = int(os.environ.get("LOCAL_WORLD_SIZE", world))
            torch.set_num_threads(max(1, (os.cpu_count() or 1) // local_world))
    if backend is None and dev.type == "cuda" and world > 1 and \
            int(os.environ.get("LOCAL_WORLD_SIZE", world)) > torch.cuda.device_count():
        # more ranks than GPUs on this node (e.g. 2 VFL parties sharing one MI355X): RCCL refuses
        # two ranks on one device, so those ranks talk over gloo (host-staged cut-layer tensors)
        backend = "gloo"
    backend = backend or ("nccl" if dev.type == "cuda" else "gloo")
    if (world > 1 or forced) and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        kw = {}
        if backend == "nccl":
            kw["device_id"] = dev
        dist.init_process_group(backend, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=timeout_s), **kw)
    _CTX = DistContext(rank, world, local, dev, backend if (world > 1 or forced) else "none",
                       forced_pg=forced)
    # peer-read all-reduce for small messages (runtime/ipc.py): one node, RCCL
    # backend. DDL_IPC_ALLREDUCE: "auto" (default) probes both paths once here and keeps the
    # peer-read kernel below the measured crossover; "1" forces it up to DDL_IPC_MAX_BYTES; "0" off.
    mode = os.environ.get("DDL_IPC_ALLREDUCE", "auto")
    if (world > 1 and backend == "nccl" and mode != "0"
            and int(os.environ.get("LOCAL_WORLD_SIZE", world)) == world and world <= 8):
        cap = int(os.environ.get("DDL_IPC_MAX_BYTES", str(16 << 20)))
        try:
            from .ipc import IpcAllReduce
            _CTX.ipc = IpcAllReduce(rank, world, dev, capacity=cap)
            _CTX.ipc_max_bytes = cap
            _CTX.ipc_policy = {"mode": "forced", "ipc_threshold_bytes": cap}
        except Exception as e:  # no peer mapping on this node: RCCL for everything
            _CTX.ipc, _CTX.ipc_max_bytes = None, 0
            _CTX.ipc_policy = {"mode": mode, "ipc_threshold_bytes": 0, "error": str(e)[:200]}
        if _CTX.ipc is not None and mode == "auto":
            probe_ipc_threshold(_CTX)
    return _CTX


PROBE_SIZES = (16 << 10, 64 << 10, 256 << 10, 1 << 20, 4 << 20, 8 << 20)


def _sync(dev) -> None:
    if torch.device(dev).type == "cuda":
        torch.cuda.synchronize(dev)


def _timed(run, iters: int, dev) -> float:
    """Mean ms per call of ``run`` (device events on a GPU, wall clock on the CPU)."""
    for _ in range(2):
        run()
    _sync(dev)
    if torch.device(dev).type == "cuda":
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            run()
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) / iters
    import time
    t0 = time.perf_counter()
    for _ in range(iters):
        run()
    return (time.perf_counter() - t0) * 1e3 / iters


def _agree_bad(bad: bool, dev) -> bool:
    """Collective: True on EVERY rank when any rank reports a failure."""
    flag = torch.tensor([1.0 if bad else 0.0], dtype=torch.float64, device=dev)
    dist.all_reduce(flag, op=dist.ReduceOp.MAX)
    return flag.item() != 0.0


def probe_ipc_threshold(ctx: DistContext, sizes=PROBE_SIZES, iters: int = 5) -> int:
    """Time the peer-read all-reduce against the process group's all-reduce (RCCL) at each size on
    every rank, take the slowest rank per (path, size) and keep the peer-read path up to the largest
    size below which it always won. Sets ctx.ipc_max_bytes / ctx.ipc_policy (identical on every
    rank: the decision is made on all-reduced timings) and releases the peer buffers when the
    probe fails (a working peer path stays mapped for rank-ordered reductions even at crossover 0).
    Returns the threshold in bytes.

    Every rank issues the SAME sequence of process-group collectives whatever happens on the peer
    path: per size, (1) a peer-path correctness check and (2) its timing each end in an agreed
    failure flag (MAX over ranks) before anything else runs, so a rank that sees wrong sums or a
    peer timeout leaves the loop at the same point as every other rank and the group falls back
    to RCCL for every size (no mismatched collectives)."""
    sizes = [s for s in sizes if s <= ctx.ipc.cap]
    dev = ctx.device
    times = torch.zeros(2, len(sizes), dtype=torch.float64, device=dev)
    failed, err = False, ""
    for j, nb in enumerate(sizes):
        # correctness first: a peer path that reads stale or unmapped memory must lose the probe
        # (rank + 1 summed over ranks: small integers, exact in fp32)
        bad = False
        try:
            y = torch.full((nb // 4,), float(ctx.rank + 1), dtype=torch.float32, device=dev)
            ctx.ipc.all_reduce(y)
            _sync(dev)
            want = float(ctx.world * (ctx.world + 1) // 2)
            if not bool((y == want).all()):
                bad, err = True, f"peer-read all-reduce of {nb} B returned wrong sums"
        except Exception as e:  # a peer timed out / the kernel refused
            bad, err = True, str(e)[:200]
        if _agree_bad(bad, dev):
            failed = True
            break
        x = torch.ones(nb // 4, dtype=torch.float32, device=dev)
        try:
            times[0, j] = _timed(lambda: ctx.ipc.all_reduce(x), iters, dev)
            if j == len(sizes) - 1:
                ctx.ipc.check()
        except Exception as e:
            bad, err = True, str(e)[:200]
        if _agree_bad(bad, dev):
            failed = True
            break
        times[1, j] = _timed(lambda: dist.all_reduce(x), iters, dev)
    dist.all_reduce(times, op=dist.ReduceOp.MAX)
    thr = 0
    if not failed:
        for j, nb in enumerate(sizes):
            if times[0, j] < times[1, j]:
                thr = nb
            else:
                break
    ctx.ipc_max_bytes = thr
    ctx.ipc_policy = {"mode": "auto", "ipc_threshold_bytes": thr,
                      "probe_ms": {str(nb): {"ipc": round(float(times[0, j]), 4), "rccl": round(float(times[1, j]), 4)}
                                   for j, nb in enumerate(sizes)}}
    if failed:
        ctx.ipc_policy["error"] = err or "a peer failed the probe"
        ctx.ipc.close()
        ctx.ipc = None
    # a working peer path stays mapped even when RCCL wins every all-reduce size: the ordered FedAvg
    # mean (fl/aggregate.py) uses it instead of an all-gather of W full partials
    return thr


def allreduce_path(ctx: DistContext, nbytes: int) -> str:
    """Which path a SUM all-reduce of ``nbytes`` fp32 takes under the context's policy."""
    if not ctx.is_distributed:
        return "none"
    return "ipc" if ctx.ipc is not None and nbytes <= ctx.ipc_max_bytes else ctx.backend


def context() -> DistContext:
    return _CTX if _CTX is not None else init()


_BARRIER_GEN = [0]


def _store_barrier(world: int, tag: str, timeout_s: float) -> None:
    """A barrier through the rendezvous store with a deadline. Unlike a process-group barrier it
    cannot hang when a peer died without raising here (an NCCL barrier would block until the
    watchdog's timeout, or forever with async error handling off): it raises TimeoutError."""
    import time
    store = dist.distributed_c10d._get_default_store()
    _BARRIER_GEN[0] += 1
    key = f"ddl_barrier/{tag}/{_BARRIER_GEN[0]}"
    store.add(key, 1)
    deadline = time.monotonic() + timeout_s
    while int(store.add(key, 0)) < world:
        if time.monotonic() > deadline:
            raise TimeoutError(f"store barrier {key}: peers missing after {timeout_s:.0f} s")
        time.sleep(0.005)


def shutdown():
    global _CTX
    err = None
    try:
        if _CTX is not None and _CTX.ipc is not None:
            try:
                _CTX.ipc.check()
            except Exception as e:  # raised after the collective teardown: peers must not wait on us
                err = e
            _CTX.ipc.close()  # collective: barrier before unmapping
    finally:
        if dist.is_initialized():
            # every rank reaches teardown before any rank closes its connections: a rank that exits
            # while a peer still drains a send / receive on one of the (many: one per pipeline link)
            # gloo groups can make that peer's transport thread throw (std::terminate -> SIGABRT)
            try:
                if err is None and _CTX is not None and _CTX.is_distributed:
                    _store_barrier(_CTX.world, "teardown", float(os.environ.get("DDL_TEARDOWN_TIMEOUT", "60")))
            except Exception:  # noqa: BLE001 - best effort: a dead peer must not hang teardown
                pass
            dist.destroy_process_group()
        _CTX = None
    if err is not None:
        raise err


def set_context(ctx: DistContext | None):
    global _CTX
    _CTX = ctx
