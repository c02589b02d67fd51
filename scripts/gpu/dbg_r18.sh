set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 120 python scripts/debug_r18_grads.py --halo 1 && timeout -k 10 120 python scripts/debug_r18_grads.py --halo 0 && DDL_KERNEL_LIB=abvar/stepadd.so timeout -k 10 120 python scripts/debug_r18_grads.py --halo 1
