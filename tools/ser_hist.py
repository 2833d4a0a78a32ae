#!/usr/bin/env python3
"""tools/ser_hist.py <dist> -- the serial pass's utilisation over time from a SER_HIST build
(DSM_LIB; tools/build_py_variant.sh with a script that adds the histogram block): per bin of
2048 wave-iterations, how many wave-iterations ran and their mean running lanes (of 64)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "hp-assignment-2_amd"))
import pydsm  # noqa: E402

dist = sys.argv[1]
n = 2 << 20 if dist == "evict" else 1 << 20
dev = torch.device("cuda", 0)
st = torch.cuda.current_stream(dev).cuda_stream
tr = torch.empty((n, 8, 4096), dtype=torch.int16, device=dev)
cn = torch.empty((n, 8), dtype=torch.int32, device=dev)
out = torch.empty((n, 4), dtype=torch.int64, device=dev)
cnt = torch.zeros(pydsm.NCOUNTERS, dtype=torch.int64, device=dev)
with pydsm.Engine(8, 4096) as eng:
    eng.generate_device(dist, 1, 4096, 0, n, tr.data_ptr(), cn.data_ptr(), st)
    eng.run_packed_device(tr.data_ptr(), cn.data_ptr(), n, out.data_ptr(), cnt.data_ptr(), st)
    torch.cuda.synchronize()
raw = cnt.cpu().numpy().view(np.uint64)
bins = [dict(bin=f"{2048*b}-{2048*(b+1) if b < 5 else 'end'}", wave_iters=int(raw[b]),
             mean_running_lanes=round(float(raw[6 + b]) / max(int(raw[b]), 1), 2)) for b in range(6)]
print(json.dumps(dict(dist=dist, bins=bins, iters_no_live=int(raw[12]))), flush=True)
