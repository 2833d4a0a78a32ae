#!/usr/bin/env bash
# tools/traffic_streams.sh [config] -- FETCH_SIZE / WRITE_SIZE passes (separate runs) of one
# transition step (tools/traffic_probe.py) under three schedules of the same workload, so the
# differences attribute the step's HBM traffic to its streams:
#   two    the default two-pass schedule (budget pass + serial resume, serial-form records)
#   one    DSM_BUDGET_LOG2=0: one lock-step pass, nothing suspended (traces + records + results)
#   lock   DSM_SERIAL=0: the lock-step resume (lock-step-form suspend records)
#   tp1    the default schedule's budget pass alone (ab/libdsm_tp1.so, TRAFFIC_PROBE=1)
#   tp2    ... without its serial-form record stores (ab/libdsm_tp2.so, TRAFFIC_PROBE=2)
# (tp1 / tp2: results invalid; built by EXTRA=-DTRAFFIC_PROBE=N tools/build_variant.sh tpN)
# Outputs under gpurun_out/traffic_<config>/<schedule>_{fetch,write}/ and <schedule>.json.
set -u
CFG=${1:-random}
OUT=gpurun_out/traffic_$CFG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp; cd - >/dev/null
for s in ${SCHEDULES:-two one lock tp1 tp2}; do
    case $s in
    two)  E="" ;;
    one)  E="DSM_BUDGET_LOG2=0" ;;
    lock) E="DSM_SERIAL=0" ;;
    tp1)  E="DSM_LIB=ab/libdsm_tp1.so" ;;
    tp2)  E="DSM_LIB=ab/libdsm_tp2.so" ;;
    tp1nolone) E="DSM_LIB=ab/libdsm_tp1.so DSM_LONE=0" ;;
    tp1late)   E="DSM_LIB=ab/libdsm_tp1.so DSM_LONE_MIN=2048" ;;
    esac
    for c in ${COUNTERS:-FETCH_SIZE WRITE_SIZE}; do
        k=$(echo $c | cut -d_ -f1 | tr A-Z a-z)
        ( [ -n "$E" ] && export $E; timeout -k 10 120 rocprofv3 --output-format csv --pmc $c \
            -d $OUT/${s}_$k -o ${s}_$k -- python3 tools/traffic_probe.py $CFG > $OUT/$s.json 2> $OUT/${s}_$k.log )
        rc=$?
        echo "$s $c rc=$rc"
        [ $rc -eq 0 ] || exit $rc
    done
done
