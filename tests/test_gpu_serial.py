"""GPU: the resume pass in serial form (dsm_engine.hip ser_kernel, csrc/dsm_serial.h).

The budget pass (lock-step, 8 lanes per system) suspends every system still running after
2^budget rounds; ser_kernel continues each on ONE lane, one node-action per iteration, with
the inboxes as 4-deep FIFOs continued in per-lane spill FIFOs in HBM (only an inbox beyond the
inbox limit hands the system to the 256-deep re-run from scratch).
It must be exact: per-system results, dump and final records, and counters equal the oracle's
single pass, and equal the lock-step resume pass (DSM_SERIAL=0), at budgets that suspend
systems early (inboxes still busy, many hand-offs) and late (the C3 tail), and for the
defined-deviation statuses raised inside the serial pass (ROUND_LIMIT, RING_OVERFLOW through
an inbox limit, ASSERT_FAILED for a home >= np)."""
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


@pytest.fixture(scope="module")
def orc():
    import pyoracle
    return pyoracle


def _cmp(a, b):
    a, b = res_to_u64(a), (b if b.ndim == 2 else res_to_u64(b))
    bad = np.nonzero((a != b).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} of {len(a)} systems differ; first {bad[:4]}: {a[bad[:2]]} vs {b[bad[:2]]}"


def _run(dsm, monkeypatch, np_, tr, cn, serial, blog, ring=12, records=(), setup=None):
    monkeypatch.setenv("DSM_SERIAL", "1" if serial else "0")
    monkeypatch.setenv("DSM_BUDGET_LOG2", str(blog))
    recs = {}
    with dsm.Engine(np_, tr.shape[2], ring_cap=ring, snapshots=bool(records)) as eng:
        if setup:
            setup(eng)
        res, cnt = eng.run_packed(tr, cn)
        info = eng.launch_info()
        for s in records:
            recs[s] = [eng.node_state(s, nd) for nd in range(np_)]
    return res, cnt, info, recs


@pytest.mark.parametrize("np_,dist,ring,blog", [(8, "uniform", 12, 12), (8, "uniform", 12, 9),
                                                (8, "uniform", 4, 10), (8, "evict", 12, 7),
                                                (8, "uniform", 16, 5), (4, "uniform", 12, 8),
                                                (4, "evict", 8, 6)])
def test_serial_resume_vs_oracle(dsm, orc, monkeypatch, np_, dist, ring, blog):
    n = 8192 if np_ == 8 else 16384
    tr, cn = orc.generate(np_, dist, 41, 4096, 3000, n)
    ores, _, odump, ofin = orc.run_packed(np_, tr, cn, records=True, nthreads=16)
    sample = list(range(0, n, 211))
    res, cnt, info, recs = _run(dsm, monkeypatch, np_, tr, cn, True, blog, ring, sample)
    _cmp(res, ores)
    for s in sample:
        mask = int(ores[s]["status"]) >> 8
        for nd, (d, f) in enumerate(recs[s]):
            assert np.array_equal(f, ofin[s, nd]), (s, nd)
            if (mask >> nd) & 1:
                assert np.array_equal(d, odump[s, nd]), (s, nd)
    assert cnt["resumed"] > 0 and info["budget_log2"] == blog
    assert info["resume_form"] == 2 and info["resume_blocks"] == min(info["cus"], -(-n // 384)), info
    assert info["budget_rounds"] == 1 << blog and info["ff_picked"] == 0, info
    if ring >= 12:          # deep inboxes spill instead of going to the 256-deep re-run
        assert cnt["overflow_reruns"] == 0
    assert cnt["systems"] == n and cnt["msgs"] == int(ores["msgs"].sum())
    assert cnt["instrs"] == int(ores["instrs"].sum()) and cnt["rounds"] == int(ores["rounds"].sum())
    assert cnt["sum_final_hash"] == int(ores["final_hash"].sum(dtype=np.uint64))
    assert cnt["sum_dump_hash"] == int(ores["dump_hash"].sum(dtype=np.uint64))
    assert cnt["max_rounds"] == int(ores["rounds"].max())
    # the lock-step resume pass gives the same counters (hand-offs may differ)
    res0, cnt0, _, _ = _run(dsm, monkeypatch, np_, tr, cn, False, blog, ring)
    _cmp(res0, ores)
    for k in ("msgs", "instrs", "rounds", "systems", "sum_final_hash", "sum_dump_hash", "max_rounds"):
        assert cnt0[k] == cnt[k], k


def test_serial_resume_on_hit_runs(dsm, orc, monkeypatch):
    """Hot-line traces with fast-forward off: the serial pass takes every hit as one action."""
    n = 4096
    tr, cn = orc.generate(8, "hot", 9, 4096, 0, n)
    ores, _ = orc.run_packed(8, tr, cn, nthreads=16)[:2]
    res, cnt, _, _ = _run(dsm, monkeypatch, 8, tr, cn, True, 11,
                          setup=lambda e: e.set_fast_forward(dsm.FF_OFF))
    _cmp(res, ores)
    assert cnt["resumed"] > n // 2


@pytest.mark.parametrize("limit_log2,blog", [(9, 6), (12, 10)])
def test_serial_round_limit(dsm, orc, monkeypatch, limit_log2, blog):
    n = 4096
    tr, cn = orc.generate(8, "uniform", 12, 4096, 0, n)
    orc.set_round_limit(1 << limit_log2)
    try:
        ores, _ = orc.run_packed(8, tr, cn, nthreads=16)[:2]
    finally:
        orc.set_round_limit(0)
    res, cnt, _, _ = _run(dsm, monkeypatch, 8, tr, cn, True, blog,
                          setup=lambda e: e.set_round_limit(limit_log2))
    _cmp(res, ores)
    assert cnt["status_ROUND_LIMIT"] == int(((ores["status"] & 0xFF) == 4).sum()) > 0
    assert cnt["resumed"] > 0


@pytest.mark.parametrize("cap", [2, 3, 6])
def test_serial_inbox_limit(dsm, orc, monkeypatch, cap):
    """An inbox limit below, at and above the serial FIFO depth (4): inboxes deeper than the
    FIFO continue in the spill, those that would pass the limit go to the 256-deep re-run,
    which reports RING_OVERFLOW exactly."""
    n = 4096
    tr, cn = orc.generate(8, "uniform", 13, 4096, 0, n)
    ores, _ = orc.run_packed(8, tr, cn, ring_cap=cap, nthreads=16)[:2]
    res, cnt, _, _ = _run(dsm, monkeypatch, 8, tr, cn, True, 7,
                          setup=lambda e: e.set_inbox_limit(cap))
    _cmp(res, ores)
    assert cnt["status_RING_OVERFLOW"] == int(((ores["status"] & 0xFF) == 2).sum())
    if cap <= 3:
        assert cnt["status_RING_OVERFLOW"] > 0


def test_serial_assert_home_beyond_np(dsm, orc, monkeypatch):
    """4-node device traces with instructions homed at nodes 4-7 late in the trace, so most
    asserts fire inside the serial pass (budget 2^5 rounds)."""
    import torch
    n = 4096
    tr, cn = orc.generate(4, "uniform", 17, 512, 0, n)
    rng = np.random.default_rng(3)
    for s in range(n):
        nd, i = int(rng.integers(0, 4)), int(rng.integers(40, 400))
        tr[s, nd, i] = (tr[s, nd, i] & 0x80FF) | ((0x40 + int(rng.integers(0, 64))) << 8)
    ores, _, _, ofin = orc.run_packed(4, tr, cn, records=True, nthreads=16)
    nasr = int(((ores["status"] & 0xFF) == 3).sum())
    assert nasr > 0
    monkeypatch.setenv("DSM_SERIAL", "1")
    monkeypatch.setenv("DSM_BUDGET_LOG2", "5")
    st = torch.cuda.current_stream().cuda_stream
    with dsm.Engine(4, 512, snapshots=True) as eng:
        dtr = torch.from_numpy(tr.view(np.int16)).cuda()
        dcn = torch.from_numpy(cn.view(np.int32)).cuda()
        out = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
        c = torch.zeros(pydsm.NCOUNTERS, dtype=torch.int64, device="cuda")
        eng.run_packed_device(dtr.data_ptr(), dcn.data_ptr(), n, out.data_ptr(), c.data_ptr(), st)
        torch.cuda.synchronize()
        res = out.cpu().numpy().view(dsm.RESULT_DTYPE).reshape(-1)
        cnt = dsm.counters_to_dict(c.cpu().numpy().view(np.uint64))
        for s in range(0, n, 61):
            for nd in range(4):
                assert np.array_equal(eng.node_state(s, nd)[1], ofin[s, nd]), (s, nd)
    _cmp(res, ores)
    assert cnt["status_ASSERT_FAILED"] == nasr and cnt["resumed"] > 0


@pytest.mark.parametrize("n", [1, 7, 385, 1537])
def test_serial_small_ensembles(dsm, orc, monkeypatch, n):
    """Ensembles that fill less than a CU's serial workgroup (384 lanes) or spill into a few:
    the serial grid and its inbox spill area are sized by ceil(n / 384) workgroups, and every
    system still reaches the oracle's result (budget 2^4: almost all of them resumed)."""
    tr, cn = orc.generate(8, "uniform", 23, 4096, 500, n)
    ores, _ = orc.run_packed(8, tr, cn, nthreads=8)[:2]
    res, cnt, info, _ = _run(dsm, monkeypatch, 8, tr, cn, True, 4)
    _cmp(res, ores)
    assert info["resume_form"] == 2 and info["resume_blocks"] == min(info["cus"], -(-n // 384)), info
    assert cnt["systems"] == n and cnt["resumed"] > 0


@pytest.mark.parametrize("np_,dist,lone_min,ring,icap", [
    (8, "uniform", 0, 12, 0), (8, "evict", 0, 12, 0), (8, "uniform", 256, 12, 0), (4, "uniform", 0, 12, 0),
    # the serial-form record laid out for ring 4 (overflow-prone: re-runs compose with it) and
    # ring 16 (the 264-word record), and read by the CAP build (an inbox limit between the
    # ring and 256 keeps the bench mode, so the budget pass writes the serial form)
    (8, "uniform", 0, 4, 0), (8, "uniform", 0, 16, 0), (8, "uniform", 0, 12, 64)])
def test_suspend_on_lone_is_exact(dsm, orc, monkeypatch, np_, dist, lone_min, ring, icap):
    """The budget pass suspends quiet-lone systems (DSM_LONE, checked every 8 rounds, from
    DSM_LONE_MIN rounds on) in the serial-form record; the serial pass resumes them with its
    lone-node macro-step.  Results and records equal the oracle and a run without it, and the
    suspensions are many more (every system that becomes lone early)."""
    n = 4096
    tr, cn = orc.generate(np_, dist, 13, 4096, 77, n)
    ores, _, odump, ofin = orc.run_packed(np_, tr, cn, records=True, nthreads=16)
    out = {}
    for lone in ("0", "8"):
        monkeypatch.setenv("DSM_LONE", lone)
        monkeypatch.setenv("DSM_LONE_MIN", str(lone_min))
        with dsm.Engine(np_, 4096, ring_cap=ring, snapshots=True) as eng:
            if icap:
                eng.set_inbox_limit(icap)
            res, cnt = eng.run_packed(tr, cn)
            li = eng.launch_info()
            assert li["resume_form"] == 2 and li["ring_cap"] == ring, li
            assert li["ser_cap"] == (1 if icap else 0), li
            for s in range(0, n, 83):
                mask = int(ores[s]["status"]) >> 8
                for nd in range(np_):
                    d, f = eng.node_state(s, nd)
                    assert np.array_equal(f, ofin[s, nd])
                    if (mask >> nd) & 1:
                        assert np.array_equal(d, odump[s, nd])
        _cmp(res, ores)
        assert cnt["msgs"] == int(ores["msgs"].sum())
        if ring >= 12:
            assert cnt["overflow_reruns"] == 0
        # the lone-node macro-step runs only in the default (non-CAP) serial build
        if icap:
            assert cnt["ser_macro_steps"] == 0, cnt
        elif lone == "8":
            assert cnt["ser_macro_steps"] > 0, cnt
        out[lone] = cnt
    assert out["8"]["resumed"] > out["0"]["resumed"], (out["8"]["resumed"], out["0"]["resumed"])
    assert out["8"]["sum_final_hash"] == out["0"]["sum_final_hash"]
