"""Single-node multi-rank launcher with failure detection.

Replaces the reference's ``run*.sh`` (``(sleep 1; python -u X.py $i > out$i.txt) &``, no exit-code
checks, rank numbering bugs such as run.bat starting at 1 — SURVEY Q17) with:

* ranks 0..W-1 always, each one GPU (``LOCAL_RANK`` = device), torchrun-compatible env
  (``RANK``, ``LOCAL_RANK``, ``WORLD_SIZE``, ``MASTER_ADDR=127.0.0.1``, ``MASTER_PORT``) plus the
  reference's positional ``argv[1] = rank`` when ``--rank-arg`` is given;
* per-rank logs ``out{rank}.txt`` (the reference's convention) or prefixed live output;
* monitoring: the first rank that exits non-zero (or a global ``--timeout``) takes the whole job
  down — SIGTERM to every rank's process group, SIGKILL after a grace period — so a crashed rank
  never leaves its peers hanging in a collective;
* exit status = the first failure's code (0 if all succeeded).

usage: python -m ddl25spring_amd.runtime.launch -n 4 [--log-dir D] [--timeout S] script.py args...
       python -m ddl25spring_amd.runtime.launch -n 4 -m ddl25spring_amd llm --dp 2 --pp 2
"""
from __future__ import annotations

import argparse
import os
import signal
import socket
import subprocess
import sys
import time


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_env(rank: int, world: int, port: int, base=None) -> dict:
    env = dict(base if base is not None else os.environ)
    env.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
               LOCAL_WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC (RCCL / tensor sharing)
    return env


def _stop(procs, grace: float = 10.0):
    for p in procs:
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except ProcessLookupError:
                pass
    t_end = time.time() + grace
    for p in procs:
        while p.poll() is None and time.time() < t_end:
            time.sleep(0.05)
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
            p.wait()


def launch(cmd: list[str], world: int, log_dir: str | None = None, timeout: float | None = None,
           rank_arg: bool = False, port: int | None = None, poll: float = 0.1) -> dict:
    """Run ``cmd`` on ``world`` ranks. -> {"returncode", "codes", "failed_rank", "elapsed"}."""
    port = port or free_port()
    procs, files = [], []
    t0 = time.time()
    try:
        for r in range(world):
            full = list(cmd) + ([str(r)] if rank_arg else [])
            out = None
            if log_dir is not None:
                os.makedirs(log_dir, exist_ok=True)
                out = open(os.path.join(log_dir, f"out{r}.txt"), "w")
                files.append(out)
            procs.append(subprocess.Popen(full, env=rank_env(r, world, port), stdout=out,
                                          stderr=subprocess.STDOUT if out else None,
                                          start_new_session=True))  # own process group per rank
        failed, code = None, 0
        while True:
            codes = [p.poll() for p in procs]
            bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
            if bad:
                failed, code = bad[0]
                break
            if all(c == 0 for c in codes):
                break
            if timeout is not None and time.time() - t0 > timeout:
                failed, code = -1, 124
                break
            time.sleep(poll)
        if failed is not None:
            _stop(procs)
        return {"returncode": code, "codes": [p.poll() for p in procs], "failed_rank": failed,
                "elapsed": time.time() - t0}
    finally:
        _stop(procs, grace=1.0)
        for f in files:
            f.close()


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("-n", "--nproc", type=int, default=1)
    ap.add_argument("--log-dir", default=None)
    ap.add_argument("--timeout", type=float, default=None)
    ap.add_argument("--rank-arg", action="store_true", help="append the rank as the last argv")
    ap.add_argument("--port", type=int, default=None)
    ap.add_argument("-m", "--module", action="store_true", help="run the target as a module (python -m)")
    ap.add_argument("script")
    ap.add_argument("args", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    cmd = [sys.executable, "-u"] + (["-m"] if a.module else []) + [a.script] + a.args
    res = launch(cmd, a.nproc, a.log_dir, a.timeout, a.rank_arg, a.port)
    if res["failed_rank"] is not None:
        who = "timeout" if res["failed_rank"] == -1 else f"rank {res['failed_rank']}"
        print(f"[launch] job stopped: {who} exited with {res['returncode']}; codes {res['codes']}",
              file=sys.stderr)
    return res["returncode"]


if __name__ == "__main__":
    sys.exit(main())
