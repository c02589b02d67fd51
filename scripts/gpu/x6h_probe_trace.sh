#!/bin/bash
# conv_x6h.hip timing probes measured by kernel trace (device time of convx6h_kernel only; the
# bench loop's host overhead and the weight-split / stats launches excluded).
#   PROBE_VAR / KGREP select another kernel's probes (DDL_HW_PROBE / convx6hw: 1 no LDS staging,
#   2 no MFMAs, 4 no loads). DDL_X6H_PROBE bits: 1 no weight DMA, 2 no halo loads, 4 no compute (fragment reads + MFMAs)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=${T:-x6hp}
#   VARS="cur notr": library variants (cur = the in-tree library, else abvar/<name>.so)
for V in ${VARS:-cur}; do
if [ "$V" = cur ]; then unset DDL_KERNEL_LIB; else export DDL_KERNEL_LIB=abvar/$V.so; fi
for cfg in ${CFGS:-"fwd:c128" "fwd:c64" "dgrad:c64" "fwd:c256"}; do
  # cfg = mode:layer[:extra bench args, comma-separated]
  IFS=: read -r M L XA <<< "$cfg"; XA=${XA//,/ }; tag=$(echo "$XA" | tr -d ' -' | tr '/' '_')
  for P in ${PROBES:-0 1 2 4 3 7}; do
    d=gpurun_out/${T}_${V}_${M}_${L}${tag}_$P
    env ${PROBE_VAR:-DDL_X6H_PROBE}=$P timeout -k 10 90 rocprofv3 --kernel-trace -d $d -o run -- python scripts/conv_f32_bench.py --mode $M --layer $L --G 8 --reps 20 $XA > $d.log 2>&1 || { echo "[$M $L $P] failed"; tail -5 $d.log; exit 1; }
    db=$(ls $d/*/run_results.db $d/run_results.db 2>/dev/null | head -1)
    echo "$V $M $L $XA probe=$P $(python scripts/prof_summary.py $db --top 8 | grep "${KGREP:-convx6h}" | head -1)"
    rm -rf $d
  done
done
done
