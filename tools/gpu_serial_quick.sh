#!/usr/bin/env bash
# serial resume: GPU tests, then C3 A/B against the lock-step resume and a budget sweep
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc; }
step ser_tests 400 python -u -m pytest tests/test_gpu_serial.py -x -q --timeout 200 --timeout-method thread
step ab_serial 400 python -u tools/ab_open.py DSM_SERIAL 0,1 1048576 2 uniform
step ab_budget 500 python -u tools/ab_open.py DSM_BUDGET_LOG2 9,10,11,12 1048576 2 uniform DSM_SERIAL=1
exit 0
