#!/usr/bin/env bash
# late budget under the default budget (2^10), C3 and C5
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/ab_open.py DSM_LATE_LOG2 0,8,9 1048576 2 uniform > gpurun_out/ab_c3.log 2>&1 || exit 1
timeout -k 10 600 python -u tools/ab_open.py DSM_LATE_LOG2 0,8,9 2097152 2 evict > gpurun_out/ab_c5.log 2>&1 || exit 1
echo done
