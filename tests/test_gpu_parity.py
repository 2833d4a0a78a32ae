"""GPU parity: the gfx950 engine (libdsm.so, through the C ABI) against the golden fixtures
and the CPU oracle, bit-exact (integer state machine: no tolerance)."""
import os
import subprocess

import numpy as np
import pytest

from conftest import (GOLD, TESTS, golden_aggregate, golden_dump, golden_ensemble, golden_ensemble_recs,
                      golden_records, inputs_dir, res_to_u64)

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


@pytest.mark.parametrize("test", TESTS)
def test_shipped_tests_dumps(dsm, orc, test, summary):
    tr, cn = orc.load_test(inputs_dir(test))
    with dsm.Engine(4, 32, snapshots=True) as eng:
        res, cnt = eng.run_packed(tr, cn)
        s = summary[test]
        r = res[0]
        assert int(r["status"]) == s["status"] | (s["dumped_mask"] << 8)
        assert (int(r["rounds"]), int(r["msgs"]), int(r["instrs"])) == (s["rounds"], s["msgs"], s["instrs"])
        assert (int(r["dump_hash"]), int(r["final_hash"])) == (s["dump_hash"], s["final_hash"])
        gold = golden_records(test)
        for core in range(4):
            d, f = eng.node_state(0, core)
            assert np.array_equal(f, gold[1, core])
            assert dsm.format_dump(core, d) == golden_dump(test, core)
        assert cnt["msgs"] == s["msgs"] and cnt["systems"] == 1


def test_c2_shipped_tests_replicated(dsm, orc, summary):
    """C2: test_1..4 replicated 16384x each (65536 systems) on one GPU."""
    reps = 16384
    trs, cns, exp = [], [], []
    for test in ["test_1", "test_2", "test_3", "test_4"]:
        tr, cn = orc.load_test(inputs_dir(test))
        trs.append(np.repeat(tr, reps, axis=0))
        cns.append(np.repeat(cn, reps, axis=0))
        s = summary[test]
        exp += [[s["status"] | (s["dumped_mask"] << 8), s["rounds"], s["msgs"], s["instrs"],
                 s["dump_hash"], s["final_hash"]]] * reps
    tr, cn = np.concatenate(trs), np.concatenate(cns)
    with dsm.Engine(4, 32) as eng:
        res, cnt = eng.run_packed(tr, cn)
    _cmp(res, np.array(exp, dtype=np.uint64))
    assert cnt["systems"] == 4 * reps


ENSEMBLES = ["np8_uniform", "np8_hot", "np8_evict", "np4_uniform", "np8_uniform_far"]


@pytest.mark.parametrize("name", ENSEMBLES)
def test_ensemble_fixture_generated(dsm, name, ensemble_meta):
    m = ensemble_meta[name]
    with dsm.Engine(m["np"], 4096) as eng:
        res, cnt = eng.run_generated(m["dist"], m["seed"], m["n_instr"], m["first_sys"], m["n_sys"])
    _cmp(res, golden_ensemble(name))
    assert cnt["systems"] == m["n_sys"]
    assert cnt["msgs"] == int(res["msgs"].sum())


@pytest.mark.parametrize("name", ["np8_uniform", "np8_hot", "np4_uniform"])
def test_ensemble_fixture_packed_and_snapshots(dsm, orc, name, ensemble_meta):
    m = ensemble_meta[name]
    n = 1024
    tr, cn = orc.generate(m["np"], m["dist"], m["seed"], m["n_instr"], m["first_sys"], n)
    with dsm.Engine(m["np"], 4096, snapshots=True) as eng:
        res, _ = eng.run_packed(tr, cn)
        recs = golden_ensemble_recs(name)
        for s in range(16):
            mask = int(res[s]["status"]) >> 8
            for nd in range(m["np"]):
                d, f = eng.node_state(s, nd)
                assert np.array_equal(f, recs[s, 1, nd])
                if (mask >> nd) & 1:
                    assert np.array_equal(d, recs[s, 0, nd])
    _cmp(res, golden_ensemble(name)[:n])


@pytest.mark.parametrize("dist", ["uniform", "hot", "evict"])
def test_large_ensemble_vs_oracle(dsm, orc, dist):
    n = 131072 if dist != "hot" else 32768
    with dsm.Engine(8, 4096, type_counts=True) as eng:
        res, cnt = eng.run_generated(dist, 11, 4096, 5_000_000, n)
    ores, obt = orc.run_generated(8, dist, 11, 4096, 5_000_000, n, nthreads=16)
    _cmp(res, ores)
    assert [cnt[f"msgs_{t}"] for t in dsm.TYPE_NAMES] == [int(x) for x in obt]
    assert cnt["sum_final_hash"] == int(ores["final_hash"].sum(dtype=np.uint64))
    assert cnt["sum_dump_hash"] == int(ores["dump_hash"].sum(dtype=np.uint64))
    assert cnt["max_rounds"] == int(ores["rounds"].max())


@pytest.mark.parametrize("ring", [4, 8, 16])
def test_ring_capacity_and_overflow_rerun(dsm, orc, ring):
    """Systems that overflow the fast kernel's LDS inbox are re-run on the device with the
    reference depth 256; results must not depend on the fast ring capacity."""
    n = 16384
    with dsm.Engine(8, 4096, ring_cap=ring, type_counts=(ring != 16)) as eng:
        res, cnt = eng.run_generated("uniform", 5, 4096, 0, n)
    ores, obt = orc.run_generated(8, "uniform", 5, 4096, 0, n, nthreads=16)
    _cmp(res, ores)
    assert cnt["systems"] == n
    if ring == 4:
        assert cnt["overflow_reruns"] > 0
    if ring != 16:
        assert [cnt[f"msgs_{t}"] for t in dsm.TYPE_NAMES] == [int(x) for x in obt]
    else:
        assert all(cnt[f"msgs_{t}"] == 0 for t in dsm.TYPE_NAMES)


def test_generator_kernel_matches_oracle(dsm, orc):
    import torch
    n = 64
    for np_, dist in [(8, "uniform"), (8, "hot"), (8, "evict"), (4, "uniform")]:
        with dsm.Engine(np_, 4096) as eng:
            tr = torch.empty((n, np_, 4096), dtype=torch.int16, device="cuda")
            cn = torch.empty((n, np_), dtype=torch.int32, device="cuda")
            eng.generate_device(dist, 9, 4000, 77, n, tr.data_ptr(), cn.data_ptr(),
                                torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            g = tr.cpu().numpy().view(np.uint16)
            otr, _ = orc.generate(np_, dist, 9, 4000, 77, n)
            assert np.array_equal(g[:, :, :4000], otr)
            assert not g[:, :, 4000:].any()
            assert (cn.cpu().numpy() == 4000).all()


def test_device_entry_points_and_accumulation(dsm, orc):
    """dsm_generate_device + dsm_run_packed_device on torch-owned HBM equal the fused-
    generator path and the oracle; counters accumulate across calls."""
    import torch
    n = 8192
    st = torch.cuda.current_stream().cuda_stream
    with dsm.Engine(8, 4096) as eng:
        tr = torch.empty((n, 8, 4096), dtype=torch.int16, device="cuda")
        cn = torch.empty((n, 8), dtype=torch.int32, device="cuda")
        out = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
        cnt = torch.zeros(pydsm.NCOUNTERS, dtype=torch.int64, device="cuda")
        eng.generate_device("evict", 3, 4096, 1000, n, tr.data_ptr(), cn.data_ptr(), st)
        eng.run_packed_device(tr.data_ptr(), cn.data_ptr(), n, out.data_ptr(), cnt.data_ptr(), st)
        eng.run_packed_device(tr.data_ptr(), cn.data_ptr(), n, out.data_ptr(), cnt.data_ptr(), st)
        torch.cuda.synchronize()
        res = out.cpu().numpy().view(dsm.RESULT_DTYPE).reshape(-1)
        c = cnt.cpu().numpy().view(np.uint64)
        gres, _ = eng.run_generated("evict", 3, 4096, 1000, n)
    ores, _ = orc.run_generated(8, "evict", 3, 4096, 1000, n, nthreads=16)
    _cmp(res, ores)
    _cmp(gres, ores)
    cd = dsm.counters_to_dict(c)
    assert cd["systems"] == 2 * n
    assert cd["msgs"] == 2 * int(ores["msgs"].sum())
    assert cd["max_rounds"] == int(ores["rounds"].max())


@pytest.mark.parametrize("dist,ring,blog", [("uniform", 12, 5), ("hot", 12, 7), ("evict", 12, 3),
                                             ("uniform", 4, 6), ("uniform", 8, 12)])
def test_two_pass_schedule(dsm, orc, monkeypatch, dist, ring, blog):
    """The packed path's two-pass schedule: a budget pass suspends every system still running
    after 2^blog rounds (state to HBM), a resume pass continues it.  With tiny budgets almost
    every system is suspended mid-flight (rings holding messages, waits pending, trace chunks
    half consumed); results, records and counters must equal the oracle's single pass, and
    overflow re-runs (ring 4) must compose with suspension."""
    monkeypatch.setenv("DSM_BUDGET_LOG2", str(blog))
    monkeypatch.setenv("DSM_FF_BUDGET_LOG2", str(blog))     # the fast-forward kernel's too
    n = 4096
    tr, cn = orc.generate(8, dist, 21, 4096, 777, n)
    with dsm.Engine(8, 4096, ring_cap=ring, snapshots=True) as eng:
        res, cnt = eng.run_packed(tr, cn)
        info = eng.launch_info()
        ores, obt, odump, ofin = orc.run_packed(8, tr, cn, records=True, nthreads=16)
        for s in range(0, n, 97):
            mask = int(ores[s]["status"]) >> 8
            for nd in range(8):
                d, f = eng.node_state(s, nd)
                assert np.array_equal(f, ofin[s, nd])
                if (mask >> nd) & 1:
                    assert np.array_equal(d, odump[s, nd])
    _cmp(res, ores)
    assert info["budget_log2"] == blog
    longer = int((ores["rounds"] >= (1 << blog)).sum())
    assert cnt["resumed"] >= longer - cnt["overflow_reruns"] and cnt["resumed"] > 0
    assert info["resume_blocks"] > 0
    assert cnt["systems"] == n and cnt["msgs"] == int(ores["msgs"].sum())
    assert cnt["sum_final_hash"] == int(ores["final_hash"].sum(dtype=np.uint64))
    assert cnt["sum_dump_hash"] == int(ores["dump_hash"].sum(dtype=np.uint64))
    assert cnt["max_rounds"] == int(ores["rounds"].max())


def test_full_size_1m_random(dsm, orc):
    """C3 at full size: 1M 8-node systems, 4096 instructions per node, traces resident in
    HBM (64 GiB).  Per-system results of the HBM-trace path equal the fused-generator path
    bit for bit; aggregate counters and hash sums equal the oracle over all 1M systems."""
    import torch
    n = 1 << 20
    st = torch.cuda.current_stream().cuda_stream
    with dsm.Engine(8, 4096) as eng:
        tr = torch.empty((n, 8, 4096), dtype=torch.int16, device="cuda")
        cn = torch.empty((n, 8), dtype=torch.int32, device="cuda")
        out = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
        cnt = torch.zeros(pydsm.NCOUNTERS, dtype=torch.int64, device="cuda")
        eng.generate_device("uniform", 1, 4096, 0, n, tr.data_ptr(), cn.data_ptr(), st)
        eng.run_packed_device(tr.data_ptr(), cn.data_ptr(), n, out.data_ptr(), cnt.data_ptr(), st)
        torch.cuda.synchronize()
        res = out.cpu().numpy().view(dsm.RESULT_DTYPE).reshape(-1)
        cd = dsm.counters_to_dict(cnt.cpu().numpy().view(np.uint64))
        del tr
        torch.cuda.empty_cache()
        gres, gcnt = eng.run_generated("uniform", 1, 4096, 0, n)
    _cmp(res, res_to_u64(gres))
    ores, obt = orc.run_generated(8, "uniform", 1, 4096, 0, n, nthreads=16)
    _cmp(res, ores)
    assert cd["sum_final_hash"] == int(ores["final_hash"].sum(dtype=np.uint64))
    assert cd["sum_dump_hash"] == int(ores["dump_hash"].sum(dtype=np.uint64))
    assert cd["msgs"] == int(ores["msgs"].sum()) and cd["instrs"] == int(ores["instrs"].sum())
    # no system fell off the serial pass's queue + spill to the 256-deep re-run (exact either
    # way, but a performance cliff)
    assert cd["overflow_reruns"] == 0
    # golden prefix / suffix pinned by the reference handler text
    _cmp(res[:4096], golden_ensemble("np8_uniform"))
    _cmp(res[999_000:1_000_024], golden_ensemble("np8_uniform_far"))
    # full-size aggregates of the reference's handler text (every system, result digest)
    assert dsm.aggregate_diff(dsm.aggregate(res), golden_aggregate("random")) == []


@pytest.mark.parametrize("dist,n", [("hot", 1 << 20), ("evict", 1 << 21)])
def test_full_size_c4_c5(dsm, orc, dist, n):
    """C4 (1M hot-line systems: the plain budget pass, then the fast-forward resume; every system
    suspended at its 448-round budget) and C5 (2M eviction-heavy systems: budget pass + serial
    resume) at full size, traces resident in HBM: per-system results and the aggregate
    counters equal the oracle over every system."""
    import torch
    st = torch.cuda.current_stream().cuda_stream
    with dsm.Engine(8, 4096) as eng:
        tr = torch.empty((n, 8, 4096), dtype=torch.int16, device="cuda")
        cn = torch.empty((n, 8), dtype=torch.int32, device="cuda")
        out = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
        cnt = torch.zeros(pydsm.NCOUNTERS, dtype=torch.int64, device="cuda")
        eng.generate_device(dist, 1, 4096, 0, n, tr.data_ptr(), cn.data_ptr(), st)
        eng.run_packed_device(tr.data_ptr(), cn.data_ptr(), n, out.data_ptr(), cnt.data_ptr(), st)
        torch.cuda.synchronize()
        res = out.cpu().numpy().view(dsm.RESULT_DTYPE).reshape(-1)
        cd = dsm.counters_to_dict(cnt.cpu().numpy().view(np.uint64))
        del tr, cn
        torch.cuda.empty_cache()
    assert cd["resumed"] > 0
    ores, _ = orc.run_generated(8, dist, 1, 4096, 0, n, nthreads=16)
    _cmp(res, ores)
    assert cd["systems"] == n and cd["max_rounds"] == int(ores["rounds"].max())
    assert cd["sum_final_hash"] == int(ores["final_hash"].sum(dtype=np.uint64))
    assert cd["sum_dump_hash"] == int(ores["dump_hash"].sum(dtype=np.uint64))
    assert cd["msgs"] == int(ores["msgs"].sum()) and cd["instrs"] == int(ores["instrs"].sum())
    assert cd["rounds"] == int(ores["rounds"].sum())
    assert cd["overflow_reruns"] == 0          # none handed to the 256-deep re-run
    # full-size aggregates of the reference's handler text (every system, result digest)
    assert dsm.aggregate_diff(dsm.aggregate(res), golden_aggregate(dist)) == []


def test_cli_end_to_end(dsm, tmp_path):
    os.symlink(os.path.join(GOLD, "inputs"), tmp_path / "tests")
    for test in TESTS:
        for f in tmp_path.glob("core_*_output.txt"):
            f.unlink()
        r = subprocess.run([dsm.CLI_PATH, test], cwd=tmp_path, capture_output=True, text=True,
                           timeout=120)
        assert r.returncode == 0, r.stderr
        assert r.stdout.splitlines() == [f"Processor {n} initialized" for n in range(4)]
        for core in range(4):
            assert (tmp_path / f"core_{core}_output.txt").read_text() == golden_dump(test, core)


def test_cli_deadlock_writes_only_finished_nodes(dsm, tmp_path):
    d = tmp_path / "tests" / "dl"
    d.mkdir(parents=True)
    progs = ["RD 0x01\nRD 0x15\n", "", "RD 0x15\nRD 0x19\n", ""]
    for n, p in enumerate(progs):
        (d / f"core_{n}.txt").write_text(p)
    r = subprocess.run([dsm.CLI_PATH, "dl"], cwd=tmp_path, capture_output=True, text=True, timeout=120)
    assert r.returncode == 2
    assert sorted(f.name for f in tmp_path.glob("core_*_output.txt")) == \
        ["core_1_output.txt", "core_2_output.txt", "core_3_output.txt"]
