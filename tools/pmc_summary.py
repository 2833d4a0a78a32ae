#!/usr/bin/env python3
"""tools/pmc_summary.py <prof_dir> [kernel-substring,...] -- per-kernel averages of the rocprofv3 PMC passes and the
kernel-trace stats written by tools/profile.sh."""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
keep = sys.argv[2].split(",") if len(sys.argv) > 2 else ["sim_kernel", "gen_kernel"]
print("== kernel stats (", d, ")")
for f in glob.glob(os.path.join(d, "kt", "*kernel_stats.csv")):
    for r in csv.DictReader(open(f)):
        print(f"  {float(r['AverageNs'])/1e6:10.3f} ms x{r['Calls']:>3}  {r['Name'][:90]}")
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(d, "pmc_*", "*counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in agg.items():
    if not any(x in k for x in keep):
        continue
    print("==", k[:100])
    for c, v in sorted(cs.items()):
        print(f"  {c:24s} {sum(v)/len(v):14.4g}")
