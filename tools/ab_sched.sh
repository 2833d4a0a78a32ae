#!/usr/bin/env bash
# tools/ab_sched.sh -- two-pass schedule parameter sweep (DSM_LATE_LOG2, DSM_BUDGET_LOG2) on
# the three bench workloads, in-process (tools/ab_env.py; every variant bit-identical).
mkdir -p gpurun_out
for d in uniform hot evict; do
  n=1048576; [ $d = evict ] && n=2097152
  timeout -k 10 300 python tools/ab_env.py DSM_LATE_LOG2 8,9,10,11 $n 2 $d || exit $?
  timeout -k 10 300 python tools/ab_env.py DSM_BUDGET_LOG2 11,12,13 $n 2 $d || exit $?
done
