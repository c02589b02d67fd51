import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP kernels on device)")
    config.addinivalue_line("markers", "slow: long-running CPU test")
    # under pytest-xdist, split the CPUs between the workers: the tabular nets' tiny CPU ops
    # with every worker running all-core intra-op pools were up to 40x slower than serial
    workers = int(os.environ.get("PYTEST_XDIST_WORKER_COUNT", "0") or 0)
    if workers > 1:
        import torch
        torch.set_num_threads(max(1, (os.cpu_count() or 1) // workers))


@pytest.fixture
def cuda():
    import gc

    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from ddl25spring_amd.ops import _lib
    _lib.kernels()  # must load: no silent fallback on a GPU box
    yield torch.device("cuda")
    # collect the test's HIP graphs / streams / pools HERE, with the device idle, rather than at
    # whatever point a later test's allocation triggers the cyclic GC (inside its own graph
    # warm-up, where destroying another graph once aborted the process)
    torch.cuda.synchronize()
    gc.collect()
    torch.cuda.synchronize()
