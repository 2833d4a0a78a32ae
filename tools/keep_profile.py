#!/usr/bin/env python3
"""tools/keep_profile.py <src> <dst> -- copy a tools/profile.sh (or gpu.sh kt) output directory
from gpurun_out/ into profiles/, keeping only this library's kernels in the per-dispatch CSVs
(the HIP runtime's fill / copy kernels and torch's own kernels dropped); logs and the
kernel-stats summaries are copied whole."""
import csv
import os
import shutil
import sys

src, dst = sys.argv[1], sys.argv[2]
DROP = ("__amd_rocclr", "at::", "direct_copy_kernel", "and_kernel_cuda", "array<char*")
for root, _, files in os.walk(src):
    out = os.path.join(dst, os.path.relpath(root, src))
    os.makedirs(out, exist_ok=True)
    for f in files:
        s, d = os.path.join(root, f), os.path.join(out, f)
        if f.endswith(("_counter_collection.csv", "_kernel_trace.csv")):
            with open(s, newline="") as fi, open(d, "w", newline="") as fo:
                r = csv.DictReader(fi)
                w = csv.DictWriter(fo, fieldnames=r.fieldnames, quoting=csv.QUOTE_NONNUMERIC)
                w.writeheader()
                for row in r:
                    if not any(x in row["Kernel_Name"] for x in DROP):
                        w.writerow(row)
        else:
            shutil.copyfile(s, d)
