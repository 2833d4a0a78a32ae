#!/usr/bin/env bash
# end-of-session check: smoke, the -m gpu suite, the default bench line, C3 kernel trace
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc; }
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread
step bench_default 600 python3 -u bench.py
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_final/kt -o kt -- python3 bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/prof_final.log 2>&1 || exit $?
echo done
