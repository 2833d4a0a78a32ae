#!/usr/bin/env python3
"""tools/traffic_probe.py [config] [systems] -- one transition step of a bench workload (traces
generated on the device, then one dsm_run_packed_device), for rocprofv3 --pmc passes that
attribute the step's HBM traffic to its streams (tools/traffic_streams.sh).  Prints the run's
counters (instructions, systems resumed, dumped nodes) as JSON for the analytic stream sizes."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "hp-assignment-2_amd"))
import pydsm  # noqa: E402

DIST = {"random": "uniform", "hot": "hot", "evict": "evict"}
cfg = sys.argv[1] if len(sys.argv) > 1 else "random"
n = int(sys.argv[2]) if len(sys.argv) > 2 else (2 << 20 if cfg == "evict" else 1 << 20)
dev = torch.device("cuda", 0)
st = torch.cuda.current_stream(dev).cuda_stream
eng = pydsm.Engine(8, 4096)
tr = torch.empty((n, 8, 4096), dtype=torch.int16, device=dev)
cn = torch.empty((n, 8), dtype=torch.int32, device=dev)
out = torch.empty((n, 4), dtype=torch.int64, device=dev)
cnt = torch.zeros(pydsm.NCOUNTERS, dtype=torch.int64, device=dev)
eng.generate_device(DIST[cfg], 1, 4096, 0, n, tr.data_ptr(), cn.data_ptr(), st)
eng.run_packed_device(tr.data_ptr(), cn.data_ptr(), n, out.data_ptr(), cnt.data_ptr(), st)
torch.cuda.synchronize()
c = pydsm.counters_to_dict(cnt.cpu().numpy().view(np.uint64))
res = out.cpu().numpy().view(pydsm.RESULT_DTYPE).reshape(-1)
dumped = int(np.unpackbits((res["status"] >> 8).astype(np.uint8)).sum())   # nodes with a dump record
li = eng.launch_info()
print(json.dumps(dict(config=cfg, systems=n, instrs=c["instrs"], msgs=c["msgs"], resumed=c["resumed"],
                      dumped_nodes=dumped, ser_macro_steps=c["ser_macro_steps"],
                      budget_log2=li["budget_log2"], resume_form=li["resume_form"],
                      kernels=li["kernels"])), flush=True)
