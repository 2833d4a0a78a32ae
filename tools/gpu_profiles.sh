#!/usr/bin/env bash
# round profiles at HEAD: C3 kernel trace + PMC passes (tools/profile.sh), C4/C5 kernel
# traces, and the default bench line with its CPU baselines
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/profile.sh c3 --steps 3 --warmup 1 || exit $?
for c in hot evict; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$c/kt -o kt -- python3 bench.py --no-cpu --config $c --steps 3 --warmup 1 > gpurun_out/prof_$c.log 2>&1 || exit $?
  echo "kt $c ok"
done
timeout -k 10 600 python3 -u bench.py > gpurun_out/bench_default.log 2>&1 || exit $?
echo done
