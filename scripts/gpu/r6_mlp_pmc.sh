#!/bin/bash
# counters of the one-launch split-NN epoch kernel (clock, MFMA busy, wait breakdown), one pass each
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r6mp}
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex mlp_epoch -d $R/gpurun_out/${T}_p1 -o p1 --output-format csv -- python3 $R/scripts/mlp_epoch_prof.py --epochs 5 > $R/gpurun_out/${T}_p1.log 2>&1
echo p1 rc=$?
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA --kernel-include-regex mlp_epoch -d $R/gpurun_out/${T}_p2 -o p2 --output-format csv -- python3 $R/scripts/mlp_epoch_prof.py --epochs 5 > $R/gpurun_out/${T}_p2.log 2>&1
echo p2 rc=$?
find $R/gpurun_out/${T}_p1 $R/gpurun_out/${T}_p2 -name "*counter_collection.csv" | while read f; do python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
acc = collections.defaultdict(float); n = collections.Counter()
for r in rows:
    acc[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
disp = collections.Counter(r["Dispatch_Id"] for r in rows)
print(sys.argv[1].split("/")[-1], "dispatches", len(disp))
for k in sorted(acc): print(f"  {k}: {acc[k] / max(1, len(disp)):.4g} per dispatch")
PY
done
