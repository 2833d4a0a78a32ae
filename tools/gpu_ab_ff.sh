#!/usr/bin/env bash
# fast-forward changes: FF / status GPU tests, then C4 (and C3 as a control) A/B vs variant libs
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fastforward.py tests/test_gpu_status.py tests/test_gpu_parity.py -k "fast_forward or round_limit or hot or two_pass or status or assert" -x -q --timeout 240 --timeout-method thread > gpurun_out/ff_tests.log 2>&1 || { echo "tests failed"; exit 1; }
bash tools/ab_libs.sh hot 1048576 default "$@" > gpurun_out/ab_ff.log 2>&1 || exit 1
bash tools/ab_libs.sh uniform 1048576 default "$@" >> gpurun_out/ab_ff.log 2>&1 || exit 1
echo done
