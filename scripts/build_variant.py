"""Build an A/B variant of the kernel library: one source recompiled with extra hipcc flags (or
from another file), linked with the in-tree objects of every other source -> abvar/<name>.so, for
DDL_KERNEL_LIB=abvar/<name>.so runs on the GPU box (scripts/gpu/ab_bench.sh, x6h_probe_trace.sh).

    python scripts/build_variant.py NAME conv_x6h.hip [-DX6H_TRANSPOSE=0 ...] [--src path/to/alt.hip]
"""
from __future__ import annotations

import argparse
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from ddl25spring_amd import _build as B  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("name")
    ap.add_argument("source")
    ap.add_argument("--src", default=None, help="compile this file in place of csrc/kernels/<source>")
    a, extra = ap.parse_known_args()
    B.build_kernels()
    out = ROOT / "abvar"
    out.mkdir(exist_ok=True)
    src = Path(a.src) if a.src else B.CSRC / "kernels" / a.source
    obj = out / f"{a.name}_{Path(a.source).stem}.o"
    flags = [f"--offload-arch={B.ARCH}", "-O3", "-std=c++17", "-fPIC", f"-I{B.CSRC / 'include'}",
             "-Wno-unused-result", "-Wno-unused-value", "-munsafe-fp-atomics",
             *B.PER_FILE_FLAGS.get(a.source, []), *extra]
    subprocess.run([B._hipcc(), *flags, "-c", str(src), "-o", str(obj)], check=True)
    objs = [obj if o.stem == Path(a.source).stem else o
            for o in sorted(B.OBJDIR.glob("*.o")) if (B.CSRC / "kernels" / (o.stem + ".hip")).exists()]
    lib = out / f"{a.name}.so"
    subprocess.run([B._hipcc(), f"--offload-arch={B.ARCH}", "-shared", "-fPIC", *map(str, objs), "-o", str(lib)],
                   check=True)
    obj.unlink()
    print(lib)


if __name__ == "__main__":
    main()
