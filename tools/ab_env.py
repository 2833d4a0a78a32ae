#!/usr/bin/env python3
"""tools/ab_env.py -- interleaved in-process A/B of transition-kernel variants selected by an
environment variable read at launch time (e.g. DSM_FW=4|8), on a bench workload with traces
resident in HBM.  Checks that every variant produces the same counters and hashes.

    python tools/ab_env.py DSM_FW 4,8 [n_systems] [reps] [dist]
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
dev = torch.device("cuda", 0)
st = torch.cuda.current_stream(dev).cuda_stream
eng = pydsm.Engine(8, 4096, timing=True)
tr = torch.empty((n, 8, 4096), dtype=torch.int16, device=dev)
cn = torch.empty((n, 8), dtype=torch.int32, device=dev)
out = torch.empty((n, 4), dtype=torch.int64, device=dev)
cnt = torch.zeros(pydsm.NCOUNTERS, dtype=torch.int64, device=dev)
eng.generate_device(dist, 1, 4096, 0, n, tr.data_ptr(), cn.data_ptr(), st)
res = {v: [] for v in variants}
info = {}
ref = None
for r in range(reps):
    for v in variants:
        os.environ[var] = v
        cnt.zero_()
        eng.run_packed_device(tr.data_ptr(), cn.data_ptr(), n, out.data_ptr(), cnt.data_ptr(), st)
        ms = eng.last_kernel_ms()
        torch.cuda.synchronize()
        raw = cnt.cpu().numpy().view(np.uint64)
        c = pydsm.counters_to_dict(raw)
        if os.environ.get("DSM_PRINT_RAW"):     # probe builds: section clocks in slots 27-31
            wr = int(raw[26])
            print(f"{v}: wave_rounds {wr} section clocks/wave-round "
                  f"{[round(int(x) / max(wr, 1), 1) for x in raw[27:32]]}", flush=True)
        key = (c["msgs"], c["sum_final_hash"], c["sum_dump_hash"])
        ref = ref or key
        assert key == ref, (v, key, ref)
        res[v].append(ms)
        if raw[:5].any():       # SER_PROBE builds: serial-pass event counts per wave
            print(f"{v}: probe iterations {int(raw[0])} macro {int(raw[1])} one-action {int(raw[2])} "
                  f"chunk-miss {int(raw[3])} hand-over {int(raw[4])} wave_rounds {int(raw[26])} "
                  f"cycles macro {int(raw[5])} one-action {int(raw[6])} hand-over {int(raw[7])} "
                  f"live-lanes {int(raw[8])} lanes-not-quiet {int(raw[9])} lanes-quiet-declined {int(raw[10])} not-at-hand {int(raw[11])} "
                  f"iters-under-half-live {int(raw[12])} hand-over cycles finish / claim / start "
                  f"{int(raw[13])} / {int(raw[14])} / {int(raw[15])} (SER_PROBE 3); macro-step phases "
                  f"entry+fetch / homes' words / decide / write-back {int(raw[13])} / {int(raw[14])} / "
                  f"{int(raw[15])} / {int(raw[16])} (SER_PROBE 4)", flush=True)
        info[v] = eng.launch_info()
for v in variants:
    print(f"{var}={v} [{dist}, {n} systems]: kernel ms median {np.median(res[v]):.2f} "
          f"min {min(res[v]):.2f}  transactions/s {ref[0] / (np.median(res[v]) * 1e-3):.3e}  "
          f"msgs {ref[0]} final_hash {ref[1]:#x} ff_passes {c['ff_passes']}  "
          f"launch {info[v]}", flush=True)
