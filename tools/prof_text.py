#!/usr/bin/env python3
"""tools/prof_text.py -- run the text kernels alone (for rocprofv3): parse_kernel over the
C3 workload's core files as text (n systems), then fmt_kernel over 8M random records."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "hp-assignment-2_amd"))
import pydsm  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
dev = torch.device("cuda", 0)
st = torch.cuda.current_stream(dev).cuda_stream
eng = pydsm.Engine(8, 4096)
off = torch.zeros(n * 8 + 1, dtype=torch.int64, device=dev)
eng.generate_text_device("uniform", 1, 4096, 0, n, 0, off.data_ptr(), st)
torch.cuda.synchronize()
tb = int(off[-1].item())
txt = torch.empty(tb + 64, dtype=torch.uint8, device=dev)
eng.generate_text_device("uniform", 1, 4096, 0, n, txt.data_ptr(), off.data_ptr(), st)
tr = torch.empty((n, 8, 4096), dtype=torch.int16, device=dev)
cn = torch.empty((n, 8), dtype=torch.int32, device=dev)
ss = torch.empty((n, 8), dtype=torch.int32, device=dev)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(reps):
    eng.parse_traces_device(txt.data_ptr(), off.data_ptr(), n * 8, 4096, tr.data_ptr(), cn.data_ptr(),
                            ss.data_ptr(), st)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / reps
print(f"parse: {ms:.3f} ms, {(tb + tr.numel() * 2) / ms / 1e6:.1f} GB/s", flush=True)
del txt, tr
m = 8 << 20
recs = torch.randint(0, 256, (m, 64), dtype=torch.uint8, device=dev)
recs[:, 32:48] %= 3
recs[:, 56:60] %= 4
out = torch.empty(m * pydsm.DUMP_SLOT, dtype=torch.uint8, device=dev)
ln = torch.empty(m, dtype=torch.int32, device=dev)
e0.record()
for _ in range(reps):
    eng.format_dumps_device(recs.data_ptr(), m, out.data_ptr(), ln.data_ptr(), 1, st)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / reps
print(f"fmt: {ms:.3f} ms, {m * (64 + pydsm.DUMP_SLOT + 4) / ms / 1e6:.1f} GB/s", flush=True)
