#!/usr/bin/env bash
# parse_kernel: GPU text tests, timing (ab_parse.py), PMC passes
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_text.py -x -q --timeout 240 --timeout-method thread > gpurun_out/text_tests.log 2>&1 || { echo "tests failed"; exit 1; }
timeout -k 10 300 python -u tools/ab_parse.py 65536 5 > gpurun_out/ab_parse.log 2>&1 || exit 1
bash tools/prof_parse.sh new || exit 1
echo done
