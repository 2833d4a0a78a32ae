#!/usr/bin/env bash
# full GPU check: smoke, the -m gpu suite, bench on C4/C5, C4 budget sweep
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc; }
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread
for c in hot evict; do step bench_$c 400 python -u bench.py --config $c --steps 10 --warmup 2 --no-cpu; done
step ab_budget_hot 400 python -u tools/ab_open.py DSM_BUDGET_LOG2 12,13,14 1048576 2 hot
exit 0
