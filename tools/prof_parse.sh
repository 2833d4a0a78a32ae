#!/usr/bin/env bash
# tools/prof_parse.sh <tag> -- PMC passes over parse_kernel (tools/ab_parse.py, one rep; DSM_LIB
# selects the build): instruction mix, waits, LDS conflicts, HBM bytes
set -u
TAG=$1
OUT=gpurun_out/profp_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
R="rocprofv3 --output-format csv"
B="python3 tools/ab_parse.py 65536 1"
run() { local name=$1; shift; timeout -s KILL 120 $R -d $OUT/$name -o $name "$@" -- $B > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
run sq --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE || exit $?
run wait --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM || exit $?
run fetch --pmc FETCH_SIZE || exit $?
run write --pmc WRITE_SIZE || exit $?
