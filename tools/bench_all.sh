#!/usr/bin/env bash
# tools/bench_all.sh [steps] [warmup] -- bench.py on C3 / C4 / C5 (gpurun_out/bench_<c>.log)
S=${1:-20}; W=${2:-5}
mkdir -p gpurun_out
for c in random hot evict; do
  timeout -k 10 400 python -u bench.py --config $c --steps $S --warmup $W > gpurun_out/bench_$c.log 2>&1 || { echo "bench $c failed"; exit 1; }
  echo "bench $c ok"
done
