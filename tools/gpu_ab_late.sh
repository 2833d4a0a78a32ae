mkdir -p gpurun_out
timeout -k 10 500 python -u tools/ab_open.py DSM_LATE_LOG2 0,8,9,10,11 1048576 2 uniform > gpurun_out/ab_late.log 2>&1
