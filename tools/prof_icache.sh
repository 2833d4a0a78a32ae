#!/usr/bin/env bash
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/ic
timeout -k 10 120 rocprofv3 -L > gpurun_out/ic/avail.txt 2>&1 || true
for v in default noff3; do
  if [ $v = default ]; then unset DSM_LIB; else export DSM_LIB=ab/libdsm_$v.so; fi
  timeout -s KILL 200 rocprofv3 --output-format csv -d gpurun_out/ic/$v -o ic --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_WAIT_INST_ANY -- python3 tools/ab_env.py DSM_NONE 0 1048576 1 uniform > gpurun_out/ic/$v.log 2>&1 || exit 1
done
