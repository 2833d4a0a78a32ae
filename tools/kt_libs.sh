#!/usr/bin/env bash
# tools/kt_libs.sh <dist> <n_systems> lib... -- per-kernel times of alternative libdsm builds
# (DSM_LIB): a rocprofv3 kernel trace of tools/ab_env.py per build, one process each, into
# gpurun_out/kt_libs/<build>_<dist>/ (kt_kernel_stats.csv), to split an A/B by kernel
D=$1; N=$2; shift 2
cd /tmp && export TMPDIR=/tmp; cd - >/dev/null
mkdir -p gpurun_out/kt_libs
for L in "$@"; do
  B=$(basename "$L" .so)
  export DSM_LIB=$L
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_libs/${B}_$D -o kt \
      -- python3 tools/ab_env.py DSM_NONE 0 $N 3 $D > gpurun_out/kt_libs/${B}_$D.log 2>&1
  rc=$?; echo "$B $D rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
