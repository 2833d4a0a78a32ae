import os, sys, numpy as np, torch
sys.path.insert(0, "hp-assignment-2_amd")
import pydsm
n = 1 << 20
dev = torch.device("cuda", 0); st = torch.cuda.current_stream(dev).cuda_stream
tr = torch.empty((n, 8, 4096), dtype=torch.int16, device=dev); cn = torch.empty((n, 8), dtype=torch.int32, device=dev)
out = torch.empty((n, 4), dtype=torch.int64, device=dev); cnt = torch.zeros(pydsm.NCOUNTERS, dtype=torch.int64, device=dev)
with pydsm.Engine(8, 4096) as g:
    g.generate_device(sys.argv[1], 1, 4096, 0, n, tr.data_ptr(), cn.data_ptr(), st)
with pydsm.Engine(8, 4096, timing=True) as eng:
    for _ in range(2):
        cnt.zero_()
        eng.run_packed_device(tr.data_ptr(), cn.data_ptr(), n, out.data_ptr(), cnt.data_ptr(), st)
        torch.cuda.synchronize()
        c = pydsm.counters_to_dict(cnt.cpu().numpy().view(np.uint64))
        print(sys.argv[1], eng.last_kernel_ms(), "wave_rounds", c["wave_rounds"], "ff_passes", c["ff_passes"], "ff_steps", c["ff_steps"], "resumed", c["resumed"])
