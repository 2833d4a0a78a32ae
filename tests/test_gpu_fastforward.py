"""GPU: the hit-run fast-forward of the transition kernel (dsm_engine.hip step (4b)).

After a round in which a system sent nothing, every further round until some node issues a
sending instruction is one local hit per non-waiting node (assignment.c:607-611 RD hit,
:635-645 WR hit on M/E); the kernel applies a whole such run per step (FF_LONG).  It must be exact:
results (rounds included), records and counters equal the oracle's, and equal the kernel's
own round-by-round path (the issue-order mode, which has no fast-forward)."""
import os
import subprocess
import tempfile

import numpy as np
import pytest

from conftest import ORACLE, golden_ensemble, res_to_u64

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


@pytest.mark.parametrize("np_,dist,ring", [(8, "hot", 12), (8, "hot", 4), (4, "hot", 12),
                                            (8, "uniform", 12), (8, "evict", 8)])
def test_packed_fast_forward_vs_oracle(dsm, orc, np_, dist, ring):
    """Packed traces (budget + resume passes, fast-forward in both), records included."""
    n = 4096
    tr, cn = orc.generate(np_, dist, 17, 4096, 123, n)
    with dsm.Engine(np_, 4096, ring_cap=ring, snapshots=True) as eng:
        res, cnt = eng.run_packed(tr, cn)
        info = eng.launch_info()
        ores, _, odump, ofin = orc.run_packed(np_, tr, cn, records=True, nthreads=16)
        for s in range(0, n, 61):
            mask = int(ores[s]["status"]) >> 8
            for nd in range(np_):
                d, f = eng.node_state(s, nd)
                assert np.array_equal(f, ofin[s, nd])
                if (mask >> nd) & 1:
                    assert np.array_equal(d, odump[s, nd])
    _cmp(res, ores)
    assert cnt["msgs"] == int(ores["msgs"].sum()) and cnt["instrs"] == int(ores["instrs"].sum())
    if dist == "hot":
        assert cnt["ff_passes"] > 0 and cnt["ff_steps"] > 0
        # the trace scan picked the fast-forward pair: its kernel ran both passes' resume
        assert info["ff_picked"] == 1 and info["resume_form"] == 3, info
        assert info["resume_blocks"] == info["grid_blocks"] and info["budget_rounds"] == 448, info
    else:
        assert info["ff_picked"] == 0 and info["resume_form"] == 2, info


def test_fast_forward_equals_round_by_round(dsm, orc):
    """The issue-order mode runs every round (no fast-forward): same results, fewer rounds
    of the wave loop with it."""
    n = 2048
    tr, cn = orc.generate(8, "hot", 5, 4096, 0, n)
    with dsm.Engine(8, 4096) as eng:
        a, ca = eng.run_packed(tr, cn)
    with dsm.Engine(8, 4096, issue_trace=True) as eng:
        b, cb = eng.run_packed(tr, cn)
    assert np.array_equal(res_to_u64(a), res_to_u64(b))
    assert cb["ff_passes"] == 0 and ca["ff_passes"] > 0
    assert ca["wave_rounds"] * 2 < cb["wave_rounds"]


def test_generated_hot_golden(dsm, ensemble_meta):
    """The fused-generator path (fast-forward over generated chunks) against the golden
    fixture pinned by the reference's handler text."""
    m = ensemble_meta["np8_hot"]
    with dsm.Engine(8, 4096) as eng:
        res, cnt = eng.run_generated(m["dist"], m["seed"], m["n_instr"], m["first_sys"], m["n_sys"])
    _cmp(res, golden_ensemble("np8_hot"))
    assert cnt["ff_passes"] > 0


@pytest.mark.parametrize("limit_log2", [6, 10])
def test_round_limit_inside_hit_runs(dsm, orc, limit_log2):
    """ROUND_LIMIT at 2^k rounds: the fast-forward stops exactly at the limit (hot systems
    are mostly inside hit runs there); packed and generated paths, against the oracle."""
    n = 2048
    tr, cn = orc.generate(8, "hot", 9, 4096, 500, n)
    orc.set_round_limit(1 << limit_log2)
    try:
        ores, _, _, ofin = orc.run_packed(8, tr, cn, records=True, nthreads=16)
        gres, _ = orc.run_generated(8, "hot", 9, 4096, 500, n, nthreads=16)
    finally:
        orc.set_round_limit(0)
    assert int(((ores["status"] & 0xFF) == 4).sum()) > n // 2
    with dsm.Engine(8, 4096, snapshots=True) as eng:
        eng.set_round_limit(limit_log2)
        res, cnt = eng.run_packed(tr, cn)
        for s in range(0, n, 97):
            assert np.array_equal(eng.node_state(s, 3)[1], ofin[s, 3])
        g, _ = eng.run_generated("hot", 9, 4096, 500, n)
        assert eng.launch_info()["round_limit_log2"] == limit_log2
    _cmp(res, ores)
    _cmp(g, gres)
    assert cnt["status_ROUND_LIMIT"] == int(((ores["status"] & 0xFF) == 4).sum())
    assert cnt["max_rounds"] == 1 << limit_log2


def test_round_limit_matches_reference_text(dsm, orc):
    """The same limit on the reference's own handler text (oracle/_ref, where built)."""
    b = os.path.join(ORACLE, "_ref", "ref_lockstep_np8")
    if not os.path.exists(b):
        pytest.skip("oracle/_ref not built")
    n = 64
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "r.bin")
        subprocess.run([b, "gen", "1", "3", "4096", "0", str(n), out], check=True,
                       env=dict(os.environ, DSM_REF_ROUND_LIMIT=str(1 << 9)))
        raw = np.fromfile(out, dtype=np.uint8).reshape(n, 32 + 2 * 8 * 64)
    ref = raw[:, :32].copy().view(orc.RES_DT).reshape(-1)
    with dsm.Engine(8, 4096) as eng:
        eng.set_round_limit(9)
        res, _ = eng.run_generated("hot", 3, 4096, 0, n)
    _cmp(res, ref)


@pytest.mark.parametrize("dist", ["uniform", "hot", "evict"])
def test_fast_forward_modes_agree(dsm, orc, dist):
    """dsm_set_fast_forward: off, on and auto give the oracle's results; auto's device-side
    trace sample picks the fast-forward kernel on the hot-line workload only (its counters
    show which kernel of the pair ran)."""
    n = 4096
    tr, cn = orc.generate(8, dist, 21, 4096, 0, n)
    ores, _ = orc.run_packed(8, tr, cn, nthreads=16)[:2]
    out = {}
    with dsm.Engine(8, 4096) as eng:
        for m in (dsm.FF_OFF, dsm.FF_ON, dsm.FF_AUTO):
            eng.set_fast_forward(m)
            out[m] = eng.run_packed(tr, cn)
            _cmp(out[m][0], ores)
    off, on, auto = out[dsm.FF_OFF][1], out[dsm.FF_ON][1], out[dsm.FF_AUTO][1]
    # off: no fast-forward step ran (the serial pass's lone-node transaction steps,
    # dsm_serial.h ser_macro, are counted apart in ser_macro_steps)
    assert off["ff_steps"] == 0 and off["ff_passes"] == 0 and off["ff_sample_instrs"] == 0
    assert on["ff_sample_instrs"] == 0
    assert auto["ff_sample_instrs"] == min(n, 4096) * 8 * 256
    picked = auto["ff_sample_runs"] * 16 >= auto["ff_sample_instrs"] and auto["ff_sample_runs"] > 0
    assert picked == (dist == "hot")
    assert (auto["ff_steps"] > 0) == picked
    if dist == "hot":
        assert on["ff_passes"] > 0 and auto["ff_passes"] > 0


@pytest.mark.parametrize("dist,picked", [("hot", 1), ("uniform", 0)])
def test_one_pass_pair_reports_the_kernel_that_ran(dsm, orc, dist, picked):
    """Budget 0 (one pass) with the automatic fast-forward pair: the launch info reads the trace
    scan's verdict back, so `ff_picked` names the kernel that ran, not the host's guess; an
    empty call afterwards reports nothing launched."""
    n = 2048
    tr, cn = orc.generate(8, dist, 3, 4096, 0, n)
    with dsm.Engine(8, 4096) as eng:
        eng.set_budget(0, 0)
        res, _ = eng.run_packed(tr, cn)
        info = eng.launch_info()
        assert info["ff_picked"] == picked and info["resume_form"] == 0, info
        assert info["budget_log2"] == 0 and info["budget_rounds"] == 0, info
        # the label names the picked half of the pair: MODE 0 (fast-forward) or M_NOFF (16)
        assert info["kernels"] == f"run=sim_kernel<8, 12, 4, false, {0 if picked else 16}, 5>", info
        eng.run_packed(tr[:0], cn[:0])
        info = eng.launch_info()
        assert info["grid_blocks"] == 0 and info["ff_picked"] == 0 and info["resume_form"] == 0, info
        assert info["kernels"] == "none", info
    ores = orc.run_packed(8, tr, cn, nthreads=16)[0]
    _cmp(res, ores)


@pytest.mark.parametrize("ffb", [7, 100, 384, 1000])
def test_long_runs_end_at_ragged_trace_ends_and_budgets(dsm, orc, monkeypatch, ffb):
    """FF_LONG (dsm_engine.hip, the run past the 8-instruction window, 8 chunks per scan step)
    must stop exactly at the group's first miss, at a trace end that is not a chunk boundary
    (ragged counts) and at the budget (FF_ON: the fast-forward kernel runs the budget pass,
    thr_ff = DSM_FF_BUDGET_ROUNDS rounds, so runs are cut mid-scan): against the oracle."""
    n = 2048
    tr, cn = orc.generate(8, "hot", 33, 4096, 900, n)
    rng = np.random.default_rng(ffb)
    cn = np.minimum(cn, rng.integers(1, 4097, size=cn.shape).astype(np.uint32))
    ores = orc.run_packed(8, tr, cn, nthreads=16)[0]
    monkeypatch.setenv("DSM_FF_BUDGET_ROUNDS", str(ffb))
    with dsm.Engine(8, 4096) as eng:
        for m in (dsm.FF_ON, dsm.FF_AUTO):
            eng.set_fast_forward(m)
            res, cnt = eng.run_packed(tr, cn)
            _cmp(res, ores)
            assert cnt["ff_steps"] > 0 and cnt["ff_passes"] > 0


@pytest.mark.parametrize("n_instr", [1001, 2045])
def test_long_runs_generated_path(dsm, orc, n_instr):
    """The fused-generator kernel's long runs (chunks generated, not loaded) with a trace
    length that ends inside a chunk."""
    n = 2048
    gres, _ = orc.run_generated(8, "hot", 41, n_instr, 300, n, nthreads=16)
    with dsm.Engine(8, 4096) as eng:
        res, cnt = eng.run_generated("hot", 41, n_instr, 300, n)
    _cmp(res, gres)
    assert cnt["ff_passes"] > 0
