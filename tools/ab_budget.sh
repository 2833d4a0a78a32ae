#!/usr/bin/env bash
# tools/ab_budget.sh [VAR] [values] -- GPU session: gpu tests, then an in-process A/B of the
# two-pass schedule's knobs (DSM_BUDGET_LOG2: 0 = one pass; DSM_LATE_LOG2: 0 = no late
# budget) on C3 with traces resident in HBM.
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?
echo tests rc=$rc; tail -3 gpurun_out/t.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python tools/ab_env.py ${1:-DSM_BUDGET_LOG2} ${2:-0,11,12,13} 1048576 3
