#!/usr/bin/env bash
# fast-forward kernel PMC on C4 (instruction mix, waits)
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1; shift; timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/pmc4_$name -o pmc -- python3 tools/ab_env.py DSM_NONE 0 1048576 1 hot > gpurun_out/pmc4_$name.log 2>&1; }
run i SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES || exit 1
run w SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS || exit 1
echo done
