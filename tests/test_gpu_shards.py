"""GPU: the multi-GPU decomposition checked on one GPU, and the
asynchronous contract of the device entry points (include/dsm.h).

bench.py gives rank r the system ids [r*n, (r+1)*n) and all-reduces the 32 counters (sums
mod 2^64, max for max_rounds).  Here 4 shards run through dsm_run_*_device with their
first_sys on one GPU; the per-system results concatenate to the one-shot run's and the summed
counters, sum_dump_hash and sum_final_hash equal the one-shot counters."""
import time

import numpy as np
import pytest

from conftest import res_to_u64

import pydsm  # noqa: E402  (numpy + ctypes only; the library loads lazily)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dsm():
    import pydsm
    if pydsm.device_count() < 1:
        pytest.fail("gpu tests need a GPU (no fallback exists)")
    return pydsm


def _reduce(vecs):
    """bench.reduce_counters on host vectors."""
    tot = np.zeros(pydsm.NCOUNTERS, dtype=np.uint64)
    for v in vecs:
        tot += v
    tot[pydsm.MAX_SLOT] = max(int(v[pydsm.MAX_SLOT]) for v in vecs)
    return tot


@pytest.mark.parametrize("dist,packed", [("uniform", True), ("hot", True), ("evict", False)])
def test_four_shards_equal_one_shot(dsm, dist, packed):
    import torch
    n, shards = 32768, 4
    st = torch.cuda.current_stream().cuda_stream
    per = n // shards
    with dsm.Engine(8, 4096) as eng:
        def run(first, cnt_sys):
            out = torch.zeros((cnt_sys, 4), dtype=torch.int64, device="cuda")
            cnt = torch.zeros(pydsm.NCOUNTERS, dtype=torch.int64, device="cuda")
            if packed:
                tr = torch.empty((cnt_sys, 8, 4096), dtype=torch.int16, device="cuda")
                cn = torch.empty((cnt_sys, 8), dtype=torch.int32, device="cuda")
                eng.generate_device(dist, 3, 4096, first, cnt_sys, tr.data_ptr(), cn.data_ptr(), st)
                eng.run_packed_device(tr.data_ptr(), cn.data_ptr(), cnt_sys, out.data_ptr(),
                                      cnt.data_ptr(), st)
            else:
                eng.run_generated_device(dist, 3, 4096, first, cnt_sys, out.data_ptr(),
                                         cnt.data_ptr(), st)
            torch.cuda.synchronize()
            return (out.cpu().numpy().view(dsm.RESULT_DTYPE).reshape(-1),
                    cnt.cpu().numpy().view(np.uint64).copy())
        whole, cw = run(0, n)
        parts = [run(r * per, per) for r in range(shards)]
    cat = np.concatenate([p[0] for p in parts])
    assert np.array_equal(res_to_u64(cat), res_to_u64(whole))
    tot = _reduce([p[1] for p in parts])
    # msgs .. max_rounds and overflow re-runs are per-system facts; wave_rounds, resumed
    # (the late budget) and the fast-forward counters describe the launch
    assert np.array_equal(tot[13:26], cw[13:26])
    d = dsm.counters_to_dict(tot)
    assert d["systems"] == n
    assert d["sum_final_hash"] == int(whole["final_hash"].sum(dtype=np.uint64))
    assert d["sum_dump_hash"] == int(whole["dump_hash"].sum(dtype=np.uint64))


def test_run_packed_device_does_not_wait(dsm):
    """The packed path's two launches (budget + resume) and the rest are enqueued without a
    host wait: behind a 0.5 s device sleep on the same stream the call returns at once."""
    import torch
    n = 65536
    s = torch.cuda.current_stream()
    st = s.cuda_stream
    with dsm.Engine(8, 4096) as eng:
        tr = torch.empty((n, 8, 4096), dtype=torch.int16, device="cuda")
        cn = torch.empty((n, 8), dtype=torch.int32, device="cuda")
        out = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
        cnt = torch.zeros(pydsm.NCOUNTERS, dtype=torch.int64, device="cuda")
        eng.generate_device("uniform", 1, 4096, 0, n, tr.data_ptr(), cn.data_ptr(), st)
        eng.run_packed_device(tr.data_ptr(), cn.data_ptr(), n, out.data_ptr(), cnt.data_ptr(), st)
        torch.cuda.synchronize()
        ref = cnt.clone()
        cnt.zero_()
        t0 = time.perf_counter()                      # calibrate the device sleep
        torch.cuda._sleep(10 ** 7)
        torch.cuda.synchronize()
        per_cycle = (time.perf_counter() - t0) / 1e7
        cycles = int(min(0.5 / max(per_cycle, 1e-12), 2 ** 62))
        torch.cuda._sleep(cycles)                     # ~0.5 s of device time ahead of the run
        t0 = time.perf_counter()
        eng.run_packed_device(tr.data_ptr(), cn.data_ptr(), n, out.data_ptr(), cnt.data_ptr(), st)
        dt = time.perf_counter() - t0
        torch.cuda.synchronize()
        assert dt < 0.1, f"run_packed_device blocked the host for {dt:.3f} s"
        assert torch.equal(cnt[13:25], ref[13:25])
        assert eng.launch_info()["resume_blocks"] > 0
