#!/usr/bin/env bash
# C4: fast-forward probe interval variants
mkdir -p gpurun_out
bash tools/ab_libs.sh hot 1048576 default "$@" > gpurun_out/ab_probe.log 2>&1 || exit 1
bash tools/ab_libs.sh hot 1048576 default "$@" >> gpurun_out/ab_probe.log 2>&1 || exit 1
echo done
