#!/usr/bin/env bash
# A/B on C3 and C5 (and C4): this build vs variant libs (ab/libdsm_*.so) + serial GPU tests
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_serial.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ser_tests.log 2>&1 || { echo "tests failed"; exit 1; }
bash tools/ab_libs.sh uniform 1048576 default "$@" > gpurun_out/ab_ser.log 2>&1 || exit 1
bash tools/ab_libs.sh evict 2097152 default "$@" >> gpurun_out/ab_ser.log 2>&1 || exit 1
bash tools/ab_libs.sh hot 1048576 default "$@" >> gpurun_out/ab_ser.log 2>&1 || exit 1
echo done
