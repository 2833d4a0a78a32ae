#!/usr/bin/env bash
# parse_kernel A/B: default vs variant libs, plus a bank-conflict PMC pass of each
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/ab_parse.log
for L in default "$@"; do
  if [ "$L" = default ]; then unset DSM_LIB; else export DSM_LIB=$L; fi
  timeout -k 10 300 python -u tools/ab_parse.py 65536 5 >> gpurun_out/ab_parse.log 2>&1 || exit 1
  n=$(basename "$L" .so)
  timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES --output-format csv -d gpurun_out/pp_$n -o pp -- python3 tools/ab_parse.py 65536 1 > gpurun_out/pp_$n.log 2>&1 || exit 1
done
echo done
