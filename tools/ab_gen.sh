#!/usr/bin/env bash
# tools/ab_gen.sh lib... -- trace-generator (gen_kernel) A/B: bench.py's trace_stream phase
# per build, interleaved twice ("default" = the tree's build).
mkdir -p gpurun_out
for r in 1 2; do for L in default "$@"; do
  if [ "$L" = default ]; then unset DSM_LIB; else export DSM_LIB=$L; fi
  timeout -k 10 300 python bench.py --no-cpu --no-dump --parse-systems 0 --steps 2 --warmup 1 > gpurun_out/abgen.log 2>&1 || { tail -5 gpurun_out/abgen.log; exit 1; }
  python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/abgen.log') if l.startswith('{')][-1]); t=d['trace_stream']; print('$L', t['ms'], t['achieved_gbs'], d['sum_final_hash'], d['roofline']['kernel_ms_avg'])"
done; done
