#!/usr/bin/env python3
"""tools/tail_probe.py <dist> [systems] -- when the budget pass's waves end, from a
SIM_TAILPROBE build (DSM_LIB=ab/libdsm_tail.so; results exact, timing not the default's):
a histogram of wave end times (ms after the wave started) that the probe build leaves in the
counter slots msgs_by_type 0-11, and the mean wave lifetime (slot 12, 10-ns ticks); the
serial pass's wave end times in slots 34-39 and its wave iterations (ser_iterations, slot 33).  A wide
spread of end times is the budget pass's tail: SIMDs idle while its last waves finish."""
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
with pydsm.Engine(8, 4096, timing=True) as eng:
    eng.generate_device(dist, 1, 4096, 0, n, tr.data_ptr(), cn.data_ptr(), st)
    for rep in range(int(os.environ.get('REPS', '2'))):
        cnt.zero_()
        eng.run_packed_device(tr.data_ptr(), cn.data_ptr(), n, out.data_ptr(), cnt.data_ptr(), st)
        ms = eng.last_kernel_ms()
        torch.cuda.synchronize()
        raw = cnt.cpu().numpy().view(np.uint64)
        waves = int(raw[:12].sum())
        bins = {"<14": int(raw[0])}
        bins.update({f"{13 + k}-{14 + k}": int(raw[k]) for k in range(1, 11)})
        bins[">=24"] = int(raw[11])
        ser = {"<11": int(raw[34])}
        ser.update({f"{10 + k}-{11 + k}": int(raw[34 + k]) for k in range(1, 5)})
        ser[">=15"] = int(raw[39])
        print(json.dumps({"dist": dist, "systems": n, "rep": rep, "kernel_ms": round(ms, 3),
                          "waves": waves, "mean_wave_ms": round(int(raw[12]) / max(waves, 1) / 1e5, 3),
                          "end_ms_hist": bins, "ser_iterations": int(raw[33]),
                          "ser_wave_rounds_total": int(raw[26]), "ser_end_ms_hist": ser,
                          "resumed": int(raw[27]), "msgs": int(raw[13]),
                          # SIM_TAILPROBE=2 builds: the serial pass's longest system and the
                          # system that ends last (iterations), slots 0-5
                          "ser_longest": {"iters": int(raw[0]) >> 32, "sys": int(raw[0]) & 0xFFFFFFFF},
                          "ser_last": {"end_iter": int(raw[1]) >> 32, "lone": (int(raw[1]) >> 31) & 1,
                                       "iters": int(raw[1]) & 0x7FFFFFFF},
                          "ser_systems_over_4000_iters": int(raw[2]),
                          "ser_nonlone_iters": int(raw[3]), "ser_all_iters": int(raw[4]),
                          "ser_nonlone_systems": int(raw[5]),
                          "final_hash": hex(int(raw[23]))}), flush=True)
