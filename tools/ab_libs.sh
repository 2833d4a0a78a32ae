#!/usr/bin/env bash
# tools/ab_libs.sh <dist> <n_systems> lib1 lib2 ... -- transition-kernel time of alternative
# libdsm builds (DSM_LIB; "default" = hp-assignment-2_amd/libdsm.so), one process per build,
# traces resident in HBM; every build must give the same counters and hashes (checked per
# process against its own first run)
D=$1; N=$2; shift 2
for L in "$@"; do
  if [ "$L" = default ]; then unset DSM_LIB; else export DSM_LIB=$L; fi
  timeout -k 10 300 python tools/ab_env.py DSM_NONE 0 $N 3 $D 2>&1 | grep "kernel ms\|probe" | sed "s|^|$L: |" || exit 1
done
