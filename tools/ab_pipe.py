#!/usr/bin/env python3
"""tools/ab_pipe.py [n_systems] [reps] [dist] [parts] -- one engine over the whole ensemble
against the ensemble cut into `parts` engines on as many streams (their kernels overlap where
one pass's tail leaves CUs idle); checks that the summed counters and hashes are identical."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "hp-assignment-2_amd"))
import pydsm  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
dist = sys.argv[3] if len(sys.argv) > 3 else "uniform"
parts = int(sys.argv[4]) if len(sys.argv) > 4 else 2
dev = torch.device("cuda", 0)
tr = torch.empty((n, 8, 4096), dtype=torch.int16, device=dev)
cn = torch.empty((n, 8), dtype=torch.int32, device=dev)
out = torch.empty((n, 4), dtype=torch.int64, device=dev)
st0 = torch.cuda.current_stream(dev)
with pydsm.Engine(8, 4096) as g:
    g.generate_device(dist, 1, 4096, 0, n, tr.data_ptr(), cn.data_ptr(), st0.cuda_stream)
torch.cuda.synchronize()
streams = [torch.cuda.Stream(dev) for _ in range(parts)]
engs = [pydsm.Engine(8, 4096) for _ in range(parts)]
one = pydsm.Engine(8, 4096)
cnts = [torch.zeros(pydsm.NCOUNTERS, dtype=torch.int64, device=dev) for _ in range(parts)]
c1 = torch.zeros(pydsm.NCOUNTERS, dtype=torch.int64, device=dev)
cut = [n * i // parts for i in range(parts + 1)]


def run_one():
    c1.zero_()
    one.run_packed_device(tr.data_ptr(), cn.data_ptr(), n, out.data_ptr(), c1.data_ptr(), st0.cuda_stream)


def run_parts():
    ev = torch.cuda.Event()
    ev.record(st0)
    for i in range(parts):
        streams[i].wait_event(ev)
        a, b = cut[i], cut[i + 1]
        with torch.cuda.stream(streams[i]):
            cnts[i].zero_()
            engs[i].run_packed_device(tr[a:].data_ptr(), cn[a:].data_ptr(), b - a, out[a:].data_ptr(),
                                      cnts[i].data_ptr(), streams[i].cuda_stream)
    for s in streams:
        st0.wait_stream(s)


def timeit(f):
    f()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


for r in range(2):
    a = timeit(run_one)
    b = timeit(run_parts)
    k1 = pydsm.counters_to_dict(c1.cpu().numpy().view(np.uint64))
    ks = [pydsm.counters_to_dict(c.cpu().numpy().view(np.uint64)) for c in cnts]
    ok = all(k1[k] == sum(x[k] for x in ks) % (1 << 64) for k in ("msgs", "instrs", "rounds", "sum_final_hash"))
    print(f"[{dist}, {n} systems] one engine {a:.2f} ms/step, {parts} parts on {parts} streams "
          f"{b:.2f} ms/step, counters {'identical' if ok else 'DIFFER'}", flush=True)
