mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_explore.py tests/test_gpu_parity.py -x -q --timeout 300 > gpurun_out/gpu_explore.log 2>&1; rc=$?; echo explore rc=$rc; tail -30 gpurun_out/gpu_explore.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python tools/ab_env.py DSM_NONE 0 1048576 2 > gpurun_out/ab.log 2>&1; echo ab rc=$?; cat gpurun_out/ab.log
