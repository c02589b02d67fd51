"""Summarise scripts/gpu/pmc_waits.sh: per conv kernel, the share of wave cycles spent waiting
(s_waitcnt / barrier), issue-stalled, and issuing, plus MFMA busy per CU-cycle and LDS conflicts.
usage: python scripts/pmc_waits_summary.py gpurun_out/pmcw [kernel-name-substring ...]"""
import glob
import os
import sqlite3
import sys
from collections import defaultdict

root = sys.argv[1]
pats = sys.argv[2:] or ["conv_"]
for tag in sorted({os.path.basename(d).rsplit("_p", 1)[0] for d in glob.glob(f"{root}/*_p1")}):
    acc = defaultdict(lambda: defaultdict(list))
    for db in glob.glob(f"{root}/{tag}_p*/**/*.db", recursive=True):
        c = sqlite3.connect(db)
        for name, ctr, val in c.execute("select kernel_name, counter_name, value from counters_collection"):
            if any(p in name for p in pats):
                key = name.split("(")[0].replace("void ", "").replace("conv_igemm_kernel", "k")[:70]
                acc[key][ctr].append(val)
    print(f"== {tag}")
    for k, d in acc.items():
        m = {c: sum(v) / len(v) for c, v in d.items()}
        wc = m.get("SQ_WAVE_CYCLES", 0) or 1
        print(f"  {k:70s} wait {m.get('SQ_WAIT_ANY', 0) / wc:5.2f} stall {m.get('SQ_WAIT_INST_ANY', 0) / wc:5.2f} "
              f"active {m.get('SQ_ACTIVE_INST_ANY', 0) / wc:5.2f} | mfma/busy "
              f"{m.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / max(m.get('SQ_BUSY_CYCLES', 1), 1):5.2f} "
              f"lds-stall {m.get('SQ_WAIT_INST_LDS', 0) / wc:5.2f} conf/lds "
              f"{m.get('SQ_LDS_BANK_CONFLICT', 0) / max(m.get('SQ_INSTS_LDS', 1), 1):5.2f} "
              f"vmem-active {m.get('SQ_ACTIVE_INST_VMEM', 0) / wc:5.2f} lds-active {m.get('SQ_ACTIVE_INST_LDS', 0) / wc:5.2f}"
              + (f" valu-active {m['SQ_ACTIVE_INST_VALU'] / wc:5.2f}" if "SQ_ACTIVE_INST_VALU" in m else "")
              + (f" valu/mfma insts {m['SQ_INSTS_VALU'] / max(m.get('SQ_INSTS_MFMA', 1), 1):5.2f}"
                 if "SQ_INSTS_VALU" in m else "")
              + (f" L2 hit {m['TCC_HIT_sum'] / max(m['TCC_HIT_sum'] + m.get('TCC_MISS_sum', 0), 1):5.2f}"
                 if "TCC_HIT_sum" in m else ""))
