#!/usr/bin/env bash
# tools/pmc_libs.sh <config> lib1 lib2 ... -- the SQ and wait PMC passes of one transition step
# (tools/traffic_probe.py) per alternative libdsm build (DSM_LIB; "default" = the tree's), in the
# layout tools/issue.py reads (gpurun_out/pmc_libs/<build>_<config>/pmc_sq, pmc_wait): waves per
# SIMD, VALU busy, wait fractions of each build's kernels, for a kernel-variant A/B's evidence.
set -u
CFG=$1; shift
cd /tmp && export TMPDIR=/tmp; cd - >/dev/null
for L in "$@"; do
  if [ "$L" = default ]; then unset DSM_LIB; B=default; else export DSM_LIB=$L; B=$(basename "$L" .so); fi
  OUT=gpurun_out/pmc_libs/${B}_$CFG
  mkdir -p $OUT
  timeout -k 10 150 rocprofv3 --output-format csv --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU \
      SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY GRBM_GUI_ACTIVE \
      -d $OUT/pmc_sq -o sq -- python3 tools/traffic_probe.py $CFG > $OUT/probe_sq.json 2> $OUT/sq.log
  rc=$?; echo "$B $CFG sq rc=$rc"; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 150 rocprofv3 --output-format csv --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
      SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT \
      -d $OUT/pmc_wait -o wait -- python3 tools/traffic_probe.py $CFG > $OUT/probe_wait.json 2> $OUT/wait.log
  rc=$?; echo "$B $CFG wait rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
exit 0
