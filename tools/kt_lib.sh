#!/bin/bash
# per-dispatch kernel durations of the transition kernel for a lib
export TMPDIR=/tmp
L=$1; T=$2   # lib ("" = default), tag
mkdir -p gpurun_out/kt_$T
DSM_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt_$T -o kt -- python3 tools/ab_env.py DSM_NONE 0 1048576 2 uniform > gpurun_out/kt_$T.log 2>&1
