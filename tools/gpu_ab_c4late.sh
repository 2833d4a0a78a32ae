#!/usr/bin/env bash
# C4 (hot): late budget x fast-forward budget
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ab_open.py DSM_LATE_LOG2 9,8,7 1048576 2 hot > gpurun_out/ab_c4late.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_open.py DSM_FF_BUDGET_LOG2 9,10 1048576 2 hot DSM_LATE_LOG2=8 >> gpurun_out/ab_c4late.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_open.py DSM_LATE_LOG2 9,8 1048576 2 uniform >> gpurun_out/ab_c4late.log 2>&1
echo done
