#!/usr/bin/env bash
# tools/fetch_libs.sh <config> lib... -- FETCH_SIZE and WRITE_SIZE (separate rocprofv3 passes) of
# one transition step (tools/traffic_probe.py) per alternative libdsm build (DSM_LIB; "default" =
# the tree's), into gpurun_out/fetch_libs/<build>_<config>/{fetch,write}; summed per kernel by
# tools/fetch_libs.py
set -u
CFG=$1; shift
cd /tmp && export TMPDIR=/tmp; cd - >/dev/null
for L in "$@"; do
  if [ "$L" = default ]; then unset DSM_LIB; B=default; else export DSM_LIB=$L; B=$(basename "$L" .so); fi
  OUT=gpurun_out/fetch_libs/${B}_$CFG
  mkdir -p $OUT
  for P in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 150 rocprofv3 --output-format csv --pmc $P -d $OUT/$P -o p \
        -- python3 tools/traffic_probe.py $CFG > $OUT/probe_$P.json 2> $OUT/$P.log
    rc=$?; echo "$B $CFG $P rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
exit 0
