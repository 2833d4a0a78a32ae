#!/usr/bin/env bash
# tools/profile.sh <tag> [bench args...] -- rocprofv3 kernel trace + PMC passes of bench.py.
# Run on the GPU box: outputs under gpurun_out/prof_<tag>/.  Counters are collected in
# separate passes (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass on gfx950).
set -u
TAG=$1; shift
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp; cd - >/dev/null
R="rocprofv3 --output-format csv"
B="python3 bench.py --no-cpu $*"
run() { local name=$1; shift; timeout -k 10 600 $R -d $OUT/$name -o $name "$@" -- $B > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
run kt --kernel-trace --stats || exit $?
run pmc_sq --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE || exit $?
run pmc_wait --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS || exit $?
run pmc_fetch --pmc FETCH_SIZE || exit $?
run pmc_write --pmc WRITE_SIZE || exit $?
exit 0
