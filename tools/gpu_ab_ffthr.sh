#!/usr/bin/env bash
# C4 (hot): the fast-forward kernel's budget as a round count; this build vs the previous one
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/ab_open.py DSM_FF_BUDGET_ROUNDS 0,320,352,384,416 1048576 2 hot > gpurun_out/ab_ffthr.log 2>&1 &&
bash tools/ab_libs.sh hot 1048576 default ab/libdsm_head.so >> gpurun_out/ab_ffthr.log 2>&1 &&
bash tools/ab_libs.sh uniform 1048576 default ab/libdsm_head.so >> gpurun_out/ab_ffthr.log 2>&1
echo done
