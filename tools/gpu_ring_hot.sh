#!/usr/bin/env bash
# C4 (hot): inbox ring depth of the lock-step kernel
mkdir -p gpurun_out
for r in 12 8 16 12; do
  timeout -k 10 300 python -u bench.py --config hot --ring $r --steps 5 --warmup 1 --no-cpu > gpurun_out/ring_$r.log 2>&1 || exit 1
  tail -1 gpurun_out/ring_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ring', $r, d['ms_per_step'], d['roofline']['kernel_ms_avg'])"
done
