"""Seeded schedule exploration and the issue-order trace (8f-3) on the CPU:
the oracle's restatement against the reference's OWN handler text driven under the same
perturbed schedules (tests/golden/explore, oracle/_ref/ref_lockstep_np4_i32) and against the
reference's own DEBUG_INSTR issue lines (:595-598); then the outcome coverage of the
exploration against the dumps the unmodified OpenMP binary produced (tests/golden/observed)."""
import hashlib
import json
import os

import numpy as np
import pytest

import pyoracle as orc
from conftest import GOLD, TESTS, inputs_dir, res_to_u64


@pytest.fixture(scope="module")
def meta():
    with open(os.path.join(GOLD, "explore", "issue_md5.json")) as f:
        return json.load(f)


def _md5(s):
    return hashlib.md5(s.encode()).hexdigest()


@pytest.mark.parametrize("test", TESTS)
def test_lockstep_issue_order_equals_reference_debug_instr(test):
    tr, cn = orc.load_test(inputs_dir(test))
    res, _, _, ev, evn = orc.run_packed_ex(4, tr, cn, issue=True)
    want = open(os.path.join(GOLD, "lockstep", test, "instruction_order.txt")).read()
    assert orc.issue_lines(ev[0, :evn[0]]) == want
    assert evn[0] == res[0]["instrs"]


@pytest.mark.parametrize("test", TESTS)
def test_oracle_exploration_equals_reference_text(test, meta):
    k = meta["k"]
    tr, cn = orc.load_test(inputs_dir(test))
    res, _, _, ev, evn = orc.run_packed_ex(4, np.repeat(tr, k, 0), np.repeat(cn, k, 0),
                                           sched_seed=meta["seed"], sched_thresh=meta["thresh"],
                                           issue=True)
    gold = np.load(os.path.join(GOLD, "explore", f"{test}.npy"))
    assert np.array_equal(res_to_u64(res), gold)
    for i in range(k):
        assert _md5(orc.issue_lines(ev[i, :evn[i]])) == meta["issue_md5"][test][i], i
    # the perturbation really explores: more than one outcome where the reference had several
    assert len({int(x) for x in res["dump_hash"]}) > (1 if test in ("sample", "test_3", "test_4") else 0)


def test_exploration_reproduces_observed_openmp_outcomes():
    """Every dump outcome the unmodified OpenMP binary produced for tests/sample is reached by
    1024 explored schedules, and nearly all explored outcomes lie in the observed sets."""
    k = 1024
    for test in ("sample", "test_1", "test_2"):
        tr, cn = orc.load_test(inputs_dir(test))
        res, dump, _, _, _ = orc.run_packed_ex(4, np.repeat(tr, k, 0), np.repeat(cn, k, 0),
                                               sched_seed=7, sched_thresh=0x8000)
        with open(os.path.join(GOLD, "observed", f"{test}.json")) as f:
            obs = json.load(f)["cores"]
        for c in range(4):
            got = {}
            for i in range(k):
                m = _md5(orc.format_dump(c, dump[i, c])) if (int(res[i]["status"]) >> 8 >> c) & 1 else "MISSING"
                got[m] = got.get(m, 0) + 1
            observed = set(obs[str(c)]["outcomes"])
            assert observed <= set(got), (test, c)
            inside = sum(v for m, v in got.items() if m in observed)
            assert inside >= 0.9 * k, (test, c, inside)
