#!/usr/bin/env bash
# serial resume: GPU tests, C3 A/B against the lock-step resume, then the C3 bench line
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc; }
step ser_tests 400 python -u -m pytest tests/test_gpu_serial.py tests/test_gpu_parity.py -k "serial or two_pass" -x -q --timeout 200 --timeout-method thread
step ab_serial 400 python -u tools/ab_open.py DSM_SERIAL 0,1 1048576 2 uniform
step bench_random 400 python -u bench.py --steps 10 --warmup 2 --no-cpu
exit 0
