#!/usr/bin/env bash
# tools/ab_quick.sh [libs...] -- transition-kernel A/B of the tree's build against the given
# alternative builds (abtmp/libdsm_<name>.so), interleaved twice, no test run first.
mkdir -p gpurun_out
L="default $*"
bash tools/ab_lib.sh $L $L
