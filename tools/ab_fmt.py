#!/usr/bin/env python3
"""tools/ab_fmt.py -- A/B of fmt_kernel tiles (DSM_FMT=16|8|4) on n random node records;
checks every variant writes identical text.  Prints GB/s (64 B read + slot + 4 B written)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "hp-assignment-2_amd"))
import pydsm  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8 << 20
variants = (sys.argv[2] if len(sys.argv) > 2 else "16,8,116,108").split(",")
reps = 5
dev = torch.device("cuda", 0)
st = torch.cuda.current_stream(dev)
g = torch.Generator(device=dev).manual_seed(1)
recs = torch.randint(0, 256, (n, 64), dtype=torch.uint8, device=dev, generator=g)
recs[:, 32:48] %= 3
recs[:, 56:60] %= 4
txt = torch.empty(n * pydsm.DUMP_SLOT, dtype=torch.uint8, device=dev)
lens = torch.empty(n, dtype=torch.int32, device=dev)
eng = pydsm.Engine(8, 8)
ref = None
for v in variants:
    os.environ["DSM_FMT"] = v
    eng.format_dumps_device(recs.data_ptr(), n, txt.data_ptr(), lens.data_ptr(), 1, st.cuda_stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        eng.format_dumps_device(recs.data_ptr(), n, txt.data_ptr(), lens.data_ptr(), 1, st.cuda_stream)
    e1.record(st)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    chk = (int(txt.view(torch.int64).sum().item()), int(lens.sum().item()))
    ref = ref or chk
    assert chk == ref, (v, chk, ref)
    b = n * (64 + pydsm.DUMP_SLOT + 4)
    print(f"DSM_FMT={v}: {ms:.3f} ms  {b / ms / 1e6:.1f} GB/s  ({b / ms / 1e6 / 8000:.3f} of 8 TB/s)", flush=True)
