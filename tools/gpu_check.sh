#!/usr/bin/env bash
# tools/gpu_check.sh -- one GPU session: smoke, gpu tests, short bench (+ optional profile).
# Stops at the first step that faults / aborts / times out (rc > 1).
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc; }
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step gpu_tests 900 python -m pytest tests -m gpu -q -rf
step bench 400 python bench.py --steps 5 --warmup 1
if [ "${PROFILE:-0}" = 1 ]; then bash tools/profile.sh ${TAG:-r01} --steps 3 --warmup 1 || exit $?; fi
exit 0
