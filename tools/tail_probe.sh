for n in 262144 524288 1048576 2097152; do timeout -k 10 300 python tools/ab_env.py DSM_NONE 0 $n 2 2>&1 | grep "kernel ms"; done
