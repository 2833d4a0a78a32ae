#!/usr/bin/env python3
"""tools/ab_parse.py [systems] [reps] -- time parse_kernel (DSM_LIB / DSM_PARSE_BPL select the
build and window) on the bench's synthetic C3 core files; checks parity with gen_kernel."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "hp-assignment-2_amd"))
import pydsm  # noqa: E402

ps = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
NP, NI = 8, 4096
dev = torch.device("cuda", 0)
sp = torch.cuda.current_stream(dev).cuda_stream
eng = pydsm.Engine(NP, NI)
tr = torch.empty((ps, NP, NI), dtype=torch.int16, device=dev)
cn = torch.empty((ps, NP), dtype=torch.int32, device=dev)
eng.generate_device("uniform", 1, NI, 0, ps, tr.data_ptr(), cn.data_ptr(), sp)
off = torch.zeros(ps * NP + 1, dtype=torch.int64, device=dev)
eng.generate_text_device("uniform", 1, NI, 0, ps, 0, off.data_ptr(), sp)
torch.cuda.synchronize()
tb = int(off[-1].item())
txt = torch.empty(tb + 64, dtype=torch.uint8, device=dev)
eng.generate_text_device("uniform", 1, NI, 0, ps, txt.data_ptr(), off.data_ptr(), sp)
ptr = torch.empty((ps, NP, NI), dtype=torch.int16, device=dev)
pcn = torch.empty((ps, NP), dtype=torch.int32, device=dev)
pst = torch.empty((ps, NP), dtype=torch.int32, device=dev)
run = lambda: eng.parse_traces_device(txt.data_ptr(), off.data_ptr(), ps * NP, NI, ptr.data_ptr(),
                                      pcn.data_ptr(), pst.data_ptr(), sp)
run()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(reps):
    run()
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / reps
ok = int(pst.abs().sum().item()) == 0 and torch.equal(pcn, cn) and torch.equal(ptr, tr)
b = tb + ptr.numel() * 2 + pcn.numel() * 4 + off.numel() * 8
print(f"{os.environ.get('DSM_LIB', 'default')} bpl={os.environ.get('DSM_PARSE_BPL', '32')}: "
      f"{ms:.3f} ms  {b / ms / 1e6:.1f} GB/s  frac {b / ms / 1e6 / 8000:.3f}  parity {'ok' if ok else 'MISMATCH'}",
      flush=True)
