mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_text.py -x -q --timeout 300 > gpurun_out/gpu_text.log 2>&1; rc=$?; echo text rc=$rc; tail -5 gpurun_out/gpu_text.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python tools/prof_text.py 65536 3
