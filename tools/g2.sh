mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -q -x > gpurun_out/gpu_tests.log 2>&1; echo tests rc=$?
timeout -k 10 300 python tools/ab_env.py DSM_FW 4,8 1048576 3 > gpurun_out/ab_fw.log 2>&1; echo ab rc=$?
cat gpurun_out/ab_fw.log; tail -3 gpurun_out/gpu_tests.log
