#!/usr/bin/env bash
# A/B on C3 / C5: this build vs variant libs (ab/libdsm_*.so)
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/ab_libs.sh uniform 1048576 "$@" > gpurun_out/ab_ser.log 2>&1 || exit 1
bash tools/ab_libs.sh evict 2097152 "$@" >> gpurun_out/ab_ser.log 2>&1 || exit 1
echo done
