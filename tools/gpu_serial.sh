#!/usr/bin/env bash
# tools/gpu_serial.sh -- serial resume pass: its GPU tests, the two-pass/full-size parity tests,
# then an A/B against the lock-step resume pass and a budget sweep on C3 (gpurun_out/*.log).
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc; }
step ser_tests 400 python -u -m pytest tests/test_gpu_serial.py -x -v --timeout 200 --timeout-method thread
step parity 600 python -u -m pytest tests/test_gpu_parity.py -x -v -k "two_pass or full_size" --timeout 300 --timeout-method thread
step ab_serial 400 python -u tools/ab_open.py DSM_SERIAL 0,1 1048576 3 uniform
step ab_budget 400 python -u tools/ab_open.py DSM_BUDGET_LOG2 10,11,12 1048576 2 uniform DSM_SERIAL=1
exit 0
