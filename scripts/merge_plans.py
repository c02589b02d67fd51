"""Merge a tuner output (scripts/conv_f32_tune.py --out X) into ddl25spring_amd/ops/f32_plans.json:
its plans replace the table's entries of the same key; with --model-prefix, the table's "blas:"
entries of the tuned geometries are dropped first (a re-tune may no longer pick the vendor GEMM).

    python scripts/merge_plans.py gpurun_out/llm_plans.json
"""
import json
import sys
from pathlib import Path

TABLE = Path(__file__).resolve().parent.parent / "ddl25spring_amd/ops/f32_plans.json"


def main():
    new = json.loads(Path(sys.argv[1]).read_text())["plans"]
    t = json.loads(TABLE.read_text())
    geoms = {k.split(":")[-1] for k in new}
    t["plans"] = {k: v for k, v in t["plans"].items() if not (k.startswith("blas:") and k.split(":")[-1] in geoms)}
    t["plans"].update(new)
    if "blas:" not in t.get("note", ""):
        t["note"] += (" 'blas:mode:...' = [vendor ms, best native ms]: the vendor fp32 GEMM was measured faster "
                      "for that plain-GEMM linear (functional_f32.vendor_gemm).")
    TABLE.write_text(json.dumps(t, indent=1))
    print(f"merged {len(new)} plans into {TABLE.name} ({len(t['plans'])} entries)")


if __name__ == "__main__":
    main()
