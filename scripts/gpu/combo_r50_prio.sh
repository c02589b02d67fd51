set -o pipefail
bash scripts/gpu/r50_fp32.sh && bash scripts/gpu/ab_env.sh DDL_GRAPH_PRIO "1 0" prio
