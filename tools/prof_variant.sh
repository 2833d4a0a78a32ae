#!/usr/bin/env bash
# tools/prof_variant.sh <tag> <VAR> <value> -- PMC passes (SQ mix + waits) of the transition
# kernel on C3 (tools/ab_env.py, one variant, one rep) for a kernel-variant A/B
set -u
TAG=$1; VAR=$2; VAL=$3
OUT=gpurun_out/profv_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
R="rocprofv3 --output-format csv"
B="python3 tools/ab_env.py $VAR $VAL 1048576 1 ${DIST:-uniform}"
run() { local name=$1; shift; timeout -k 10 300 $R -d $OUT/$name -o $name "$@" -- $B > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
run pmc_sq --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE || exit $?
run pmc_wait --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS || exit $?
