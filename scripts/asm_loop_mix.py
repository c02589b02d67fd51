"""Instruction mix of the hottest loop of a kernel in a hipcc device-assembly file.

Usage: python scripts/asm_loop_mix.py conv_f32.s <symbol-substring>

Finds the function, then every basic-block range [label, backward branch to label] and reports
the one with the most MFMAs: counts per class (MFMA, VALU, DS read/write, buffer/global, SALU,
waitcnt / barrier) and the VALU opcodes by frequency — the quickest way to see whether a kernel's
main loop is MFMA-, VALU- or LDS-issue bound before spending a GPU run (cycle costs: MI355X
microarch guide, per-instruction cycle constants).
"""
import re
import sys
from collections import Counter


def main():
    path, sym = sys.argv[1], sys.argv[2]
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l) and sym in l)
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
    body = lines[start:end]
    labels = {m.group(1): i for i, l in enumerate(body) if (m := re.match(r"^(\.LBB\S+):", l))}
    best = None
    for i, l in enumerate(body):
        m = re.match(r"\s+s_cbranch_\w+\s+(\.LBB\S+)|\s+s_branch\s+(\.LBB\S+)", l)
        if not m:
            continue
        tgt = m.group(1) or m.group(2)
        if tgt in labels and labels[tgt] < i:
            seg = body[labels[tgt]:i + 1]
            n = sum(1 for s in seg if "v_mfma" in s)
            if best is None or n > best[0]:
                best = (n, labels[tgt], i, seg)
    if best is None:
        print("no loop found")
        return
    _, a, b, seg = best
    cls = Counter()
    valu = Counter()
    for s in seg:
        t = s.strip().split()
        if not t or t[0].startswith((";", ".")) or t[0].endswith(":"):
            continue
        op = t[0]
        if op.startswith("v_mfma"):
            cls["mfma"] += 1
        elif op.startswith("v_"):
            cls["valu"] += 1
            valu[op] += 1
        elif op.startswith("ds_read") or op.startswith("ds_load"):
            cls["ds_read"] += 1
        elif op.startswith("ds_write") or op.startswith("ds_store"):
            cls["ds_write"] += 1
        elif op.startswith(("buffer_", "global_")):
            cls["vmem"] += 1
        elif op.startswith("s_waitcnt") or op == "s_barrier":
            cls[op] += 1
        elif op.startswith("s_"):
            cls["salu"] += 1
    print(f"loop lines {start + a}-{start + b}: " + ", ".join(f"{k}={v}" for k, v in cls.most_common()))
    print("VALU: " + ", ".join(f"{k}={v}" for k, v in valu.most_common(30)))


if __name__ == "__main__":
    main()
