#!/usr/bin/env bash
# ser_kernel PMC passes (waits, LDS) on C3 + variant A/B
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1; shift; timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/pmc_$name -o pmc -- python3 tools/ab_env.py DSM_NONE 0 1048576 1 uniform > gpurun_out/pmc_$name.log 2>&1; }
run w SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT || exit 1
run i SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM || exit 1
bash tools/ab_libs.sh uniform 1048576 default "$@" > gpurun_out/ab_ser.log 2>&1 || exit 1
echo done
