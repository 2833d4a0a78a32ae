#!/usr/bin/env bash
# tools/ab_reps.sh <dist> <n_systems> lib... -- tools/ab_libs.sh with 5 reps per process and two alternating rounds (noisy A/Bs)
D=$1; N=$2; shift 2
for r in 1 2; do for L in "$@"; do
  export DSM_LIB=$L
  timeout -k 10 300 python tools/ab_env.py DSM_NONE 0 $N 5 $D 2>&1 | grep "kernel ms" | sed "s|^|$L: |" | cut -c1-120 || exit 1
done; done
