#!/usr/bin/env bash
# tools/ab_gpu.sh [libs...] -- one GPU session: the gpu tests on the tree's build, then the
# transition-kernel A/B of the tree's build against the given alternative builds (twice).
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?
echo tests rc=$rc; tail -2 gpurun_out/t.log; [ $rc -le 1 ] || exit $rc
L="default $*"
bash tools/ab_lib.sh $L $L
