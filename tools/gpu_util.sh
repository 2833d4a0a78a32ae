#!/usr/bin/env bash
# instrumented serial pass (ab/libdsm_miss.so): cycles in the chunk-miss wait vs the whole loop
mkdir -p gpurun_out
DSM_LIB=ab/libdsm_miss.so timeout -k 10 300 python -u tools/lane_util.py uniform > gpurun_out/util.log 2>&1 || exit 1
DSM_LIB=ab/libdsm_miss.so timeout -k 10 300 python -u tools/lane_util.py evict >> gpurun_out/util.log 2>&1 || exit 1
