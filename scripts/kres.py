"""Register / spill / occupancy summary of every kernel in one HIP source (hipcc resource remarks).

    python scripts/kres.py csrc/kernels/conv_x6h.hip [name-filter]
"""
import re
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
src = ROOT / sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", f"-I{ROOT / 'csrc/include'}",
       "-munsafe-fp-atomics", "--cuda-device-only", "-c", str(src), "-o", "/tmp/kres.o",
       "-Rpass-analysis=kernel-resource-usage"]
err = subprocess.run(cmd, capture_output=True, text=True, cwd="/tmp").stderr
cur, out = None, {}
for line in err.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur, out = m.group(1), {}
        continue
    m = re.search(r"remark:\s+(VGPRs|VGPRs Spill|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|"
                  r"LDS Size \[bytes/block\]): (\d+)", line)
    if m and cur:
        out[m.group(1)] = m.group(2)
        if m.group(1).startswith("LDS") and flt in cur:
            print(f"{cur[:72]:72s} vgpr={out.get('VGPRs')} spill={out.get('VGPRs Spill')} "
                  f"scratch={out.get('ScratchSize [bytes/lane]')} occ={out.get('Occupancy [waves/SIMD]')} lds={m.group(2)}")
