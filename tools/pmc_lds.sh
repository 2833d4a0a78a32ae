#!/usr/bin/env bash
# tools/pmc_lds.sh <tag> [config] -- LDS and issue counters of one transition step
# (tools/traffic_probe.py; DSM_LIB selects the build) in one rocprofv3 --pmc pass.
set -u
TAG=$1; CFG=${2:-random}
OUT=gpurun_out/pmc_lds_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp; cd - >/dev/null
timeout -k 10 120 rocprofv3 --output-format csv --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE \
    -d $OUT -o lds -- python3 tools/traffic_probe.py $CFG > $OUT/probe.json 2> $OUT/lds.log
rc=$?; echo "pmc_lds $TAG rc=$rc"; exit $rc
