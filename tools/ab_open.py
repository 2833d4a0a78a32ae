#!/usr/bin/env python3
"""tools/ab_open.py -- interleaved A/B of engine variants selected by an environment variable
read at dsm_open (DSM_SERIAL, DSM_BUDGET_LOG2, DSM_LATE_LOG2, ...), or VAR=FF for the
fast-forward mode (0 off, 1 on, 2 auto: dsm_set_fast_forward): a fresh engine per variant
per repetition, traces generated once and resident in HBM; checks that every variant gives
the same counters and hashes.

    python tools/ab_open.py VAR v1,v2,.. [n_systems] [reps] [dist] [VAR2=val ...]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "hp-assignment-2_amd"))
import pydsm  # noqa: E402

var = sys.argv[1]
variants = sys.argv[2].split(",")
n = int(sys.argv[3]) if len(sys.argv) > 3 else 1 << 20
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 3
dist = sys.argv[5] if len(sys.argv) > 5 else "uniform"
for kv in sys.argv[6:]:
    k, v = kv.split("=", 1)
    os.environ[k] = v
dev = torch.device("cuda", 0)
st = torch.cuda.current_stream(dev).cuda_stream
tr = torch.empty((n, 8, 4096), dtype=torch.int16, device=dev)
cn = torch.empty((n, 8), dtype=torch.int32, device=dev)
out = torch.empty((n, 4), dtype=torch.int64, device=dev)
cnt = torch.zeros(pydsm.NCOUNTERS, dtype=torch.int64, device=dev)
with pydsm.Engine(8, 4096) as g:
    g.generate_device(dist, 1, 4096, 0, n, tr.data_ptr(), cn.data_ptr(), st)
res = {v: [] for v in variants}
ctr = {}
ref = None
for r in range(reps):
    for v in variants:
        if var != "FF":
            os.environ[var] = v
        with pydsm.Engine(8, 4096, timing=True) as eng:
            if var == "FF":
                eng.set_fast_forward(int(v))
            cnt.zero_()
            eng.run_packed_device(tr.data_ptr(), cn.data_ptr(), n, out.data_ptr(), cnt.data_ptr(), st)
            torch.cuda.synchronize()
            ms = eng.last_kernel_ms()
        c = pydsm.counters_to_dict(cnt.cpu().numpy().view(np.uint64))
        key = (c["msgs"], c["sum_final_hash"], c["sum_dump_hash"], c["rounds"])
        ref = ref or key
        assert key == ref, (v, key, ref)
        res[v].append(ms)
        ctr[v] = {k: c[k] for k in ("resumed", "overflow_reruns", "wave_rounds")}
        print(f"  rep {r} {var}={v}: {ms:.2f} ms", flush=True)
for v in variants:
    print(f"{var}={v} [{dist}, {n} systems]: kernel ms median {np.median(res[v]):.2f} "
          f"min {min(res[v]):.2f}  transactions/s {ref[0] / (np.median(res[v]) * 1e-3):.3e}  {ctr[v]}",
          flush=True)
