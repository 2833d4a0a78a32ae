#!/usr/bin/env bash
# tools/prof_text.sh <tag> -- rocprofv3 kernel trace + PMC passes of tools/prof_text.py
set -u
TAG=$1
OUT=gpurun_out/prof_text_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
R="rocprofv3 --output-format csv"
B="python3 tools/prof_text.py 65536 2"
run() { local name=$1; shift; timeout -k 10 300 $R -d $OUT/$name -o $name "$@" -- $B > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
run kt --kernel-trace --stats || exit $?
run pmc_sq --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE || exit $?
run pmc_wait --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS || exit $?
run pmc_fetch --pmc FETCH_SIZE || exit $?
run pmc_write --pmc WRITE_SIZE || exit $?
exit 0
