#!/usr/bin/env python3
"""tools/ab_occ.py -- interleaved in-process A/B of transition-kernel variants (DSM_OCC)
on the bench workload (C3, traces resident in HBM).  Prints per-variant kernel ms."""
import os
import sys
import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "hp-assignment-2_amd"))
import pydsm  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
variants = [int(v) for v in (sys.argv[2].split(",") if len(sys.argv) > 2 else ["1", "4", "5", "6"])]
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
dist = sys.argv[4] if len(sys.argv) > 4 else "uniform"
dev = torch.device("cuda", 0)
st = torch.cuda.current_stream(dev).cuda_stream
eng = pydsm.Engine(8, 4096, timing=True)
tr = torch.empty((n, 8, 4096), dtype=torch.int16, device=dev)
cn = torch.empty((n, 8), dtype=torch.int32, device=dev)
out = torch.empty((n, 4), dtype=torch.int64, device=dev)
cnt = torch.zeros(32, dtype=torch.int64, device=dev)
eng.generate_device(dist, 1, 4096, 0, n, tr.data_ptr(), cn.data_ptr(), st)
res = {v: [] for v in variants}
ref = None
for r in range(reps):
    for v in variants:
        os.environ["DSM_OCC"] = str(v)
        cnt.zero_()
        eng.run_packed_device(tr.data_ptr(), cn.data_ptr(), n, out.data_ptr(), cnt.data_ptr(), st)
        ms = eng.last_kernel_ms()
        torch.cuda.synchronize()
        c = pydsm.counters_to_dict(cnt.cpu().numpy().view(np.uint64))
        key = (c["msgs"], c["sum_final_hash"], c["sum_dump_hash"])
        ref = ref or key
        assert key == ref, (v, key, ref)
        res[v].append(ms)
for v in variants:
    print(f"DSM_OCC={v}: kernel ms median {np.median(res[v]):.2f} min {min(res[v]):.2f}  "
          f"msgs/s {ref[0] / (np.median(res[v]) * 1e-3):.3e}  launch {eng.launch_info()['waves_per_cu']}")
