#!/usr/bin/env bash
# C4 kernel trace at HEAD
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_hot/kt -o kt -- python3 bench.py --no-cpu --config hot --steps 3 --warmup 1 > gpurun_out/prof_hot.log 2>&1 || exit $?
echo done
