#!/usr/bin/env python3
"""tools/traffic_table.py <dir> -- per-kernel FETCH_SIZE / WRITE_SIZE (bytes per dispatch,
summed over the dispatch's rows) of tools/traffic_streams.sh's schedules, plus the probe's
counters, as JSON on stdout."""
import collections
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
out = {}
for s in ("two", "one", "lock", "tp1", "tp2", "tp1nolone", "tp1late"):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for k in ("fetch", "write"):
        for f in glob.glob(os.path.join(d, f"{s}_{k}", "*counter_collection.csv")):
            for r in csv.DictReader(open(f)):
                name = r["Kernel_Name"].replace("void (anonymous namespace)::", "").split("(")[0]
                disp = r.get("Dispatch_Id", "")
                per[(name, disp)][r["Counter_Name"]] += float(r["Counter_Value"]) * 1024.0
    agg = collections.defaultdict(lambda: dict(FETCH_SIZE=0.0, WRITE_SIZE=0.0, dispatches=0))
    for (name, disp), cs in per.items():
        for c, v in cs.items():
            agg[name][c] += v
        agg[name]["dispatches"] += 1
    try:
        meta = json.loads(open(os.path.join(d, f"{s}.json")).read().strip().splitlines()[-1])
    except (OSError, ValueError, IndexError):
        meta = {}
    out[s] = dict(meta=meta, kernels={k: {c: int(v) if c != "dispatches" else v for c, v in x.items()}
                                       for k, x in sorted(agg.items())})
print(json.dumps(out, indent=1))
