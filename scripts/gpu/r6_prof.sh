#!/bin/bash
# rocprofv3 kernel trace of a python script: scripts/gpu/r6_prof.sh TAG script.py [args]
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
T=$1; shift
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$T -o run -- python "$@" > gpurun_out/prof_$T.log 2>&1
rc=$?
tail -5 gpurun_out/prof_$T.log
f=$(find gpurun_out/prof_$T -name '*kernel_trace.csv' | head -1)
[ -n "$f" ] && python - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[-60:]:
    print(r["Kernel_Name"][:60], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
PY
exit $rc
