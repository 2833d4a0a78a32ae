#!/usr/bin/env python3
"""tools/ser_probe.py <dist> [systems] -- the serial pass's diagnostic counters of a SER_PROBE
build (DSM_LIB=ab/libdsm_serprobe*.so; results of such a build are exact, its timing is not):
per-wave event counts and s_memtime cycle sums the probe build leaves in the counter slots
msgs_by_type 0-16 (dsm_engine.hip ser_kernel, SER_PROBE)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "hp-assignment-2_amd"))
import pydsm  # noqa: E402

dist = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else (2 << 20 if dist == "evict" else 1 << 20)
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
names = ["iters", "iters_macro", "iters_one_action", "iters_chunk_miss", "iters_handover",
         "cyc_macro_phase", "cyc_one_action_phase", "cyc_handover_phase", "live_lanes",
         "lanes_not_quiet", "lanes_quiet_declined", "lanes_instr_not_at_hand", "iters_lt32_live",
         "cyc13", "cyc14", "cyc15", "cyc16"]
print(json.dumps({k: int(raw[i]) for i, k in enumerate(names)}), flush=True)
