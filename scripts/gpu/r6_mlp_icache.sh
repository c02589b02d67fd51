#!/bin/bash
# instruction-cache counters of the one-launch split-NN epoch kernel
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r6ic}
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc ${PMC:-SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE GRBM_GUI_ACTIVE} --kernel-include-regex mlp_epoch -d $R/gpurun_out/${T}_p1 -o p1 --output-format csv -- python3 $R/scripts/mlp_epoch_prof.py --epochs 5 > $R/gpurun_out/${T}_p1.log 2>&1
echo p1 rc=$?
find $R/gpurun_out/${T}_p1 -name "*counter_collection.csv" | while read f; do python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
acc = collections.defaultdict(float)
for r in rows:
    acc[r["Counter_Name"]] += float(r["Counter_Value"])
disp = collections.Counter(r["Dispatch_Id"] for r in rows)
print(sys.argv[1].split("/")[-1], "dispatches", len(disp))
for k in sorted(acc): print(f"  {k}: {acc[k] / max(1, len(disp)):.4g} per dispatch")
PY
done
tail -3 $R/gpurun_out/${T}_p1.log
