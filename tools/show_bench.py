#!/usr/bin/env python3
"""tools/show_bench.py [log...] -- one summary line per bench.py JSON line."""
import glob
import json
import sys

for f in sys.argv[1:] or sorted(glob.glob("gpurun_out/bench_*.log")):
    lines = [l for l in open(f) if l.startswith("{")]
    if not lines:
        print(f, "no JSON")
        continue
    d = json.loads(lines[-1])
    km = d.get("kernel_ms") or [0]
    cb, cp = d.get("cpu_baseline") or {}, d.get("cpu_port") or {}
    print(f"{f}: {d['value'] / 1e9:.2f} Gtx/s  {d['ms_per_step']} ms/step  kernel {sum(km) / len(km):.2f} ms  "
          f"frac {d['roofline']['frac']}  cpu {cb.get('value', 0) / 1e9:.3f} ({cb.get('kind')}, {cb.get('cores')} thr)  "
          f"port {cp.get('value', 0) / 1e9:.3f}  gen {(d.get('trace_stream') or {}).get('frac')}  "
          f"parse {(d.get('trace_parse') or {}).get('frac')}  fmt {(d.get('dump_stream') or {}).get('frac')}  "
          f"ff {d['counters'].get('ff_passes')}/{d['counters'].get('ff_steps')}")
