"""GPU schedule exploration (dsm_set_schedule) and issue-order trace
(DSM_F_ISSUE_TRACE, 8f-3) through the C ABI: bit-exact against the reference's own handler
text under the same perturbed schedules (tests/golden/explore), its DEBUG_INSTR lines, and
the oracle on generated ensembles."""
import hashlib
import json
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLD, TESTS, inputs_dir, res_to_u64

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dsm():
    import pydsm
    if pydsm.device_count() < 1:
        pytest.fail("gpu tests need a GPU (no fallback exists)")
    return pydsm


@pytest.fixture(scope="module")
def meta():
    with open(os.path.join(GOLD, "explore", "issue_md5.json")) as f:
        return json.load(f)


def _md5(s):
    return hashlib.md5(s.encode()).hexdigest()


@pytest.mark.parametrize("test", TESTS)
def test_gpu_issue_order_lockstep_equals_reference(dsm, test):
    import pyoracle as orc
    tr, cn = orc.load_test(inputs_dir(test))
    with dsm.Engine(4, 32, issue_trace=True) as eng:
        res, _ = eng.run_packed(tr, cn)
        ev = eng.issue_trace(0)
    assert len(ev) == int(res[0]["instrs"])
    want = open(os.path.join(GOLD, "lockstep", test, "instruction_order.txt")).read()
    assert dsm.format_issue_trace(ev) == want


@pytest.mark.parametrize("test", TESTS)
def test_gpu_exploration_equals_reference_text(dsm, test, meta):
    import pyoracle as orc
    k = meta["k"]
    tr, cn = orc.load_test(inputs_dir(test))
    with dsm.Engine(4, 32, issue_trace=True) as eng:
        eng.set_schedule(meta["seed"], meta["thresh"])
        res, _ = eng.run_packed(np.repeat(tr, k, 0), np.repeat(cn, k, 0))
        md5s = [_md5(dsm.format_issue_trace(eng.issue_trace(i))) for i in range(k)]
    assert np.array_equal(res_to_u64(res), np.load(os.path.join(GOLD, "explore", f"{test}.npy")))
    assert md5s == meta["issue_md5"][test]


@pytest.mark.parametrize("dist,thresh", [("uniform", 0x8000), ("hot", 0x4000), ("evict", 0xC000)])
def test_gpu_exploration_generated_vs_oracle(dsm, dist, thresh):
    """8-node generated ensembles under three act thresholds; both the packed-trace and the
    fused-generator engine paths equal the oracle's exploration bit for bit."""
    import pyoracle as orc
    n, n_instr = 2048, 512
    tr, cn = orc.generate(8, dist, 3, n_instr, 0, n)
    ores, _, _, oev, oevn = orc.run_packed_ex(8, tr, cn, sched_seed=11, sched_thresh=thresh,
                                              issue=True)
    with dsm.Engine(8, n_instr, issue_trace=True) as eng:
        eng.set_schedule(11, thresh)
        res, _ = eng.run_packed(tr, cn)
        for i in (0, 1, 777, n - 1):
            assert np.array_equal(eng.issue_trace(i), oev[i, :oevn[i]]), i
        gres, _ = eng.run_generated(dist, 3, n_instr, 0, n)
        eng.set_schedule(0, dsm.SCHED_LOCKSTEP)
        lres, _ = eng.run_packed(tr, cn)
    assert np.array_equal(res_to_u64(res), res_to_u64(ores))
    assert np.array_equal(res_to_u64(gres), res_to_u64(ores))
    lo, _, _, _, _ = orc.run_packed_ex(8, tr, cn)
    assert np.array_equal(res_to_u64(lres), res_to_u64(lo))
    assert not np.array_equal(res_to_u64(lres), res_to_u64(res))


def test_cli_issue_order_and_schedule(dsm, tmp_path):
    os.symlink(os.path.join(GOLD, "inputs"), tmp_path / "tests")
    r = subprocess.run([dsm.CLI_PATH, "--issue-order", "order.txt", "test_1"], cwd=tmp_path,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert (tmp_path / "order.txt").read_text() == \
        open(os.path.join(GOLD, "lockstep", "test_1", "instruction_order.txt")).read()
    # an explored schedule of tests/sample: its dumps are one of the reference's observed outcomes
    with open(os.path.join(GOLD, "observed", "sample.json")) as f:
        obs = json.load(f)["cores"]
    r = subprocess.run([dsm.CLI_PATH, "--schedule", "7:32768", "sample"], cwd=tmp_path,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    for c in range(4):
        assert _md5((tmp_path / f"core_{c}_output.txt").read_text()) in obs[str(c)]["outcomes"]


def test_gpu_exploration_with_inbox_overflow_rerun(dsm):
    """ring 4 overflows: those systems re-run in the 256-deep kernel under the same explored
    schedule (the stall hash depends on system, round and node only) -- still bit-exact."""
    import pyoracle as orc
    n = 8192
    tr, cn = orc.generate(8, "uniform", 5, 1024, 0, n)
    ores, _, _, _, _ = orc.run_packed_ex(8, tr, cn, sched_seed=5, sched_thresh=0xA000)
    with dsm.Engine(8, 1024, ring_cap=4, type_counts=True) as eng:
        eng.set_schedule(5, 0xA000)
        res, cnt = eng.run_packed(tr, cn)
    assert cnt["overflow_reruns"] > 0
    assert np.array_equal(res_to_u64(res), res_to_u64(ores))
    assert cnt["msgs"] == int(ores["msgs"].sum())
