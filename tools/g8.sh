mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_text.py -x -q --timeout 300 > gpurun_out/gpu_simc.log 2>&1; rc=$?; echo tests rc=$rc; tail -30 gpurun_out/gpu_simc.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python tools/ab_env.py DSM_SIMC 0,1 1048576 2 > gpurun_out/ab_simc.log 2>&1; echo ab rc=$?; cat gpurun_out/ab_simc.log
timeout -k 10 300 python tools/ab_env.py DSM_SIMC_RING 10,12 1048576 2 > gpurun_out/ab_ring.log 2>&1; echo ab rc=$?; cat gpurun_out/ab_ring.log
