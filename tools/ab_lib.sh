#!/usr/bin/env bash
# tools/ab_lib.sh lib1 lib2 ... -- time the transition kernel of alternative libdsm builds
# (DSM_LIB) on C3, one process per build; "default" = hp-assignment-2_amd/libdsm.so
for L in "$@"; do
  if [ "$L" = default ]; then unset DSM_LIB; else export DSM_LIB=$L; fi
  timeout -k 10 300 python tools/ab_env.py DSM_NONE 0 1048576 2 2>&1 | grep "kernel ms" | sed "s|^|$L: |" || exit 1
done
