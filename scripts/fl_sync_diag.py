"""Where does the bf16 unsynchronised-rounds spread come from? (VERDICT r4 correctness debt 7a)

tests/test_fl_gpu.py::test_unsynchronised_rounds_match_on_device trains MnistCnn (bf16 path) for
3 FedAvg rounds synchronised, unsynchronised and synchronised again. This script repeats each mode
several times in ONE process (so every instance shares the autotuner's cached picks, which it also
prints) plus a "jittered" synchronised mode that only perturbs launch timing (a spin kernel on the
stream before each round), and prints every run's distance to the first synchronised run relative
to a round's update. If the unsynchronised runs land as far from the synchronised ones as jittered
synchronised runs do, the spread is timing-dependent fp32-atomic order (split-K WGRAD) amplified by
bf16 rounding — not an ordering / plan / buffer-reuse bug in the unsynchronised path (which the
fp32 path checks bit for bit: test_fp32_gpu.py::test_fp32_unsynchronised_rounds_equal_exactly).

    python scripts/fl_sync_diag.py [--reps 3] [--modes sync,unsync,unsync_s,jitter]

"unsync_s" runs the unsynchronised code path with a device sync after every round: if it matches
the synchronised runs while "unsync" does not, the difference is a cross-stream race exposed by the
host running ahead, not a code-path difference.
"""
from __future__ import annotations

import argparse
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from ddl25spring_amd.data.images import DeviceImageDataset, synthetic_images  # noqa: E402
from ddl25spring_amd.data.split import split  # noqa: E402
from ddl25spring_amd.fl.algorithms import FedAvg  # noqa: E402
from ddl25spring_amd.models import mnist_cnn  # noqa: E402
from ddl25spring_amd.ops import autotune  # noqa: E402
from ddl25spring_amd.runtime.dist import DistContext  # noqa: E402


def run(mode: str, cuda):
    arr = synthetic_images("mnist", 800, seed=0)
    parts = split(4, True, 3, labels=arr.labels)
    fa = FedAvg(mnist_cnn, DeviceImageDataset(arr, cuda), parts, lr=0.05, batch_size=50,
                client_fraction=1.0, seed=3, ctx=DistContext(device=cuda), eval_every=0)
    w0 = fa.w_global.clone()
    fa.round()
    fa.sync_rounds = not mode.startswith("unsync")
    for i in range(3):
        if mode == "jitter":
            torch.cuda._sleep(int(2e5 * (1 + i)))  # perturb launch timing only
        fa.round()
        if mode == "unsync_s":  # unsynchronised code path, but the host never runs ahead
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    return w0, fa.w_global.clone(), len(autotune.cache())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--modes", default="sync,unsync,jitter")
    a = ap.parse_args()
    cuda = torch.device("cuda")
    ref = prev = None
    for rep in range(a.reps):
        for mode in a.modes.split(","):
            w0, w, ntune = run(mode, cuda)
            if ref is None:
                ref, step = w, (w - w0).norm()
                print(f"rep {rep} {mode:6s}: reference (update norm {step.item():.4e}), tuner keys {ntune}")
                prev = w
                continue
            rel = ((w - ref).norm() / step).item()
            same_prev = prev is not None and torch.equal(w, prev)
            print(f"rep {rep} {mode:6s}: rel to first run {rel:.3e}  bitwise {torch.equal(w, ref)}  "
                  f"equal to previous run {same_prev}  tuner keys {ntune}", flush=True)
            prev = w


if __name__ == "__main__":
    main()
