#!/usr/bin/env python3
"""tools/asm_blocks.py <file.s> <kernel-substring> -- per basic block of one kernel in a
hipcc -S listing: VALU / SALU / LDS / VMEM instruction counts and the loop depth comment, to
see where a kernel's instructions sit (static counts, not executed counts)."""
import re
import sys

src, want = sys.argv[1], sys.argv[2]
lines = open(src).read().splitlines()
start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*%s\S*:" % re.escape(want), l))
blocks, cur = [], None
for l in lines[start:]:
    if l.startswith("\t.end_amdhsa_kernel") or l.startswith(".Lfunc_end"):
        break
    m = re.match(r"^(\.LBB\w+|; %bb\.\d+):(.*)$", l)
    if m or cur is None:
        cur = dict(name=m.group(1) if m else "entry", note=(m.group(2).strip() if m else ""),
                   v=0, s=0, d=0, g=0)
        blocks.append(cur)
        if m:
            continue
    t = l.strip()
    if t.startswith(";") and "Loop" in t and not cur["note"]:
        cur["note"] = t
    ins = t.split()[0] if t and not t.startswith(";") and not t.startswith(".") else ""
    if ins.startswith("v_"):
        cur["v"] += 1
    elif ins.startswith("s_"):
        cur["s"] += 1
    elif ins.startswith("ds_"):
        cur["d"] += 1
    elif ins.startswith(("global_", "buffer_", "scratch_", "flat_")):
        cur["g"] += 1
tot = dict(v=0, s=0, d=0, g=0)
for b in blocks:
    for k in tot:
        tot[k] += b[k]
    if b["v"] + b["s"] + b["d"] + b["g"]:
        print(f"{b['name']:12s} v{b['v']:4d} s{b['s']:4d} ds{b['d']:3d} mem{b['g']:3d}  {b['note'][:70]}")
print("total", tot)
