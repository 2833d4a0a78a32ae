#!/usr/bin/env python3
"""tools/fetch_libs.py [dir] -- per build and kernel, the FETCH_SIZE / WRITE_SIZE (KB units,
summed over the kernel's dispatches and rows) of tools/fetch_libs.sh's passes, in GB (raw)."""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/fetch_libs"
for b in sorted(glob.glob(os.path.join(d, "*"))):
    out = {}
    for p in ("FETCH_SIZE", "WRITE_SIZE"):
        tot = collections.Counter()
        for f in glob.glob(os.path.join(b, p, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"].split("::")[-1].split("<")[0].split("(")[0]
                tot[k] += float(r["Counter_Value"]) * 1024
        out[p] = {k: round(v / 1e9, 3) for k, v in tot.items() if v > 1e7}
    print(os.path.basename(b), out)
