"""ASan + UBSan build of the native host runtime (csrc/runtime/runtime.cpp), driven by
csrc/tests/runtime_sanitize.cpp over every exported entry point (sanitizers).

Host code only: GPU AddressSanitizer / xnack+ code objects are not available on the target pool, so
the device kernels are covered by their numerics tests instead. Skipped if g++ lacks libasan."""
import os
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


@pytest.mark.timeout(300)
def test_runtime_under_asan_ubsan(tmp_path):
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("g++ not available")
    exe = tmp_path / "rt_san"
    cmd = [cxx, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer",
           "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
           str(ROOT / "csrc/runtime/runtime.cpp"), str(ROOT / "csrc/tests/runtime_sanitize.cpp"),
           "-o", str(exe), "-pthread"]
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        if "asan" in res.stderr.lower() or "ubsan" in res.stderr.lower():
            pytest.skip("sanitizer runtime libraries unavailable: " + res.stderr[-300:])
        raise AssertionError(res.stderr)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    run = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=240)
    assert run.returncode == 0, run.stdout + run.stderr
    assert "runtime sanitize ok" in run.stdout
