#!/usr/bin/env bash
# tools/gpu_round.sh -- smoke, the -m gpu suite, then bench.py on C3/C4/C5 (gpurun_out/*.log).
# Stops at the first step that faults / aborts / times out (rc > 1).
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc; }
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread
for c in random hot evict; do step bench_$c 400 python -u bench.py --config $c --steps ${STEPS:-10} --warmup 2 --no-cpu; done
exit 0
