#!/usr/bin/env python3
"""tools/traffic.py <prof_dir> <config> -- HBM traffic per launch from the rocprofv3
FETCH_SIZE / WRITE_SIZE passes (separate runs, KB units) written by tools/profile.sh, folded
into profiles/pmc_traffic.json under <config> for bench.py's roofline "traffic" fields.

gfx950 correction (MI355X_MICROARCH.md, HBM): FETCH_SIZE reports 1/2 of the bytes of a wide
coalesced 16-B-per-lane streaming read, so fetch is doubled for kernels whose loads are of
that shape (parse_kernel, fmt_kernel's template copies); WRITE_SIZE is exact for 16-B-per-lane
streaming stores.  The transition kernel's 16-B per-lane chunk loads are scattered across
nodes (uncalibrated): its traffic is the doubled fetch plus writes, with the raw value kept."""
import collections
import csv
import glob
import json
import os
import sys

d, config = sys.argv[1], sys.argv[2]
KERNELS = {"sim_kernel": "::sim_kernel<", "ser_kernel": "::ser_kernel<", "gen_kernel": "::gen_kernel<",
           "parse_kernel": "::parse_kernel<", "fmt_kernel": "::fmt_kernel<"}
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(d, "pmc_fetch", "*counter_collection.csv")) + \
        glob.glob(os.path.join(d, "pmc_write", "*counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        for k, pat in KERNELS.items():
            if pat in r["Kernel_Name"] and "256, 1," not in r["Kernel_Name"]:
                vals[k][(r["Counter_Name"], r.get("Dispatch_Id", r.get("Correlation_Id", "")))].append(
                    float(r["Counter_Value"]))
out = {}
for k, v in vals.items():
    per = collections.defaultdict(list)
    for (cname, _disp), xs in v.items():
        per[cname].append(sum(xs) * 1024.0)       # KB -> bytes, summed over the dispatch's rows
    if k in ("sim_kernel", "ser_kernel", "parse_kernel"):
        # (parse_kernel: the EXACT pass over the files the FAST pass abandoned -- none for the
        # bench's generated text -- runs after each FAST pass and reads nothing)
        # the packed path launches a fast-forward / plain pair per pass and one of the two
        # exits at once (ffscan_kernel's verdict): average over the dispatches that ran
        per = {c: [x for x in xs if x >= (1 << 20)] or xs for c, xs in per.items()}
    fetch = sum(per["FETCH_SIZE"]) / max(len(per["FETCH_SIZE"]), 1)
    write = sum(per["WRITE_SIZE"]) / max(len(per["WRITE_SIZE"]), 1)
    out[k] = dict(bytes_per_launch=int(2 * fetch + write), fetch_bytes_raw=int(fetch),
                  fetch_bytes_gfx950_x2=int(2 * fetch), write_bytes=int(write),
                  dispatches=len(per["FETCH_SIZE"]),
                  source=f"{d}/pmc_fetch + pmc_write (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, "
                         f"separate passes, KB units, fetch x2 per the gfx950 correction)")
p = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles", "pmc_traffic.json")
try:
    allv = json.load(open(p))
except (OSError, ValueError):
    allv = {}
allv[config] = out
json.dump(allv, open(p, "w"), indent=1, sort_keys=True)
print(json.dumps(out, indent=1))
