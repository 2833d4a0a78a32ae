"""Pins the CPU oracle (oracle/dsm_oracle.c) before anything is checked against it.

Golden data (tests/golden/, made by oracle/gen_fixtures.py in the build container):
  * lock-step dumps of the reference's own handler text (oracle/_ref/ref_lockstep_np4_i32),
  * their md5s, which must also equal SURVEY.md Appendix A,
  * outcome sets of the unmodified OpenMP reference binary (200 runs per test),
  * per-system results of the reference handler text over the synthetic generator.
"""
import hashlib
import json
import os

import numpy as np
import pytest

import pyoracle as orc
from conftest import (GOLD, TESTS, golden_dump, golden_ensemble, golden_ensemble_recs,
                      golden_records, inputs_dir, res_to_u64)

# lock-step dump md5s (reference handler text, independent probe)
SURVEY_MD5 = {
    "sample": ["f79b11c610f62d062d228659e281862e", "76c0ded4f51994b5b4f2289d6b61eb89",
               "2e9ab3cefc05d9efa78c81e86c7d5307", "50f83fafae3f5c26773d52920d6e91e2"],
    "test_1": ["247a200d3b970468ecdcd6a8df8eb385", "eadb0267e20c062b965be1ef8df4ca26",
               "01fec99d700cd0de5ae9fec8d61a2d14", "46a12c0cd78bf8a27930185d05ea6e0f"],
    "test_2": ["43afef8059bc97ed54eb0d3eb571ffaa", "efad5e18bf4ab5264d0fd2553c710fe3",
               "d0d33599b5d6c25af2620ce2cf6fac47", "9388d6c7807774227ba337d090b92a51"],
    "test_3": ["988fd45a603ad8bf1d993b74bc8575cb", "7bc4f39ff1d61ebe127d0b6d17377ca2",
               "69c9a207ce6c35a07b4dd890fb9d0fb1", "cfd20f6fac8c56571766069bf1a28c0f"],
    "test_4": ["7a95aec82beeb4afe81cf859c9afbd75", "d1a7cd84c26a97f307bbb911c1985f40",
               "8cc5262fcae1b3e1a58ca8e974948023", "f6342ddf1205d8f5e15cbb78c7c507e4"],
}
# rounds / messages under the lock-step schedule
SURVEY_ROUNDS_MSGS = {"sample": (9, 10), "test_1": (41, 92), "test_2": (41, 92),
                      "test_3": (30, 59), "test_4": (44, 69)}


@pytest.mark.parametrize("test", TESTS)
def test_golden_dumps_match_survey_md5(test, summary):
    for core in range(4):
        txt = golden_dump(test, core)
        assert hashlib.md5(txt.encode()).hexdigest() == SURVEY_MD5[test][core]
        assert summary[test]["md5"][str(core)] == SURVEY_MD5[test][core]
    assert (summary[test]["rounds"], summary[test]["msgs"]) == SURVEY_ROUNDS_MSGS[test]


@pytest.mark.parametrize("test", TESTS)
def test_oracle_reproduces_lockstep_dumps(test, summary):
    tr, cn = orc.load_test(inputs_dir(test))
    res, bt, dump, fin = orc.run_packed(4, tr, cn, records=True, nthreads=1)
    s = summary[test]
    r = res[0]
    assert int(r["status"]) & 0xFF == s["status"]
    assert int(r["status"]) >> 8 == s["dumped_mask"]
    assert (int(r["rounds"]), int(r["msgs"]), int(r["instrs"])) == (s["rounds"], s["msgs"], s["instrs"])
    assert (int(r["dump_hash"]), int(r["final_hash"])) == (s["dump_hash"], s["final_hash"])
    assert int(bt.sum()) == s["msgs"]
    gold = golden_records(test)
    assert np.array_equal(dump[0], gold[0]) and np.array_equal(fin[0], gold[1])
    for core in range(4):
        assert orc.format_dump(core, dump[0, core]) == golden_dump(test, core)


@pytest.mark.parametrize("test", TESTS)
def test_lockstep_outcome_is_an_observed_reference_outcome(test):
    """Schedule invariance: the lock-step dump of every core is one of the
    dumps the unmodified OpenMP reference produced, and equals it on every line that did
    not vary across the observed runs."""
    with open(os.path.join(GOLD, "observed", f"{test}.json")) as f:
        obs = json.load(f)
    for core in range(4):
        mine = golden_dump(test, core)
        outs = obs["cores"][str(core)]["outcomes"]
        assert hashlib.md5(mine.encode()).hexdigest() in outs
        texts = [o["text"].splitlines() for o in outs.values()]
        ml = mine.splitlines()
        for i in range(len(ml)):
            col = {t[i] for t in texts if i < len(t)}
            if len(col) == 1:
                assert ml[i] in col, (test, core, i)


@pytest.mark.parametrize("test", ["sample", "test_1", "test_2"])
def test_deterministic_tests_single_outcome(test):
    """sample (cores 2,3), test_1 and test_2 were schedule-independent in the reference."""
    with open(os.path.join(GOLD, "observed", f"{test}.json")) as f:
        obs = json.load(f)
    cores = [2, 3] if test == "sample" else [0, 1, 2, 3]
    for core in cores:
        outs = obs["cores"][str(core)]["outcomes"]
        assert list(outs) == [hashlib.md5(golden_dump(test, core).encode()).hexdigest()]


ENSEMBLES = ["np8_uniform", "np8_hot", "np8_evict", "np4_uniform", "np8_uniform_far"]


@pytest.mark.parametrize("name", ENSEMBLES)
def test_oracle_matches_reference_handler_text_on_ensembles(name, ensemble_meta):
    m = ensemble_meta[name]
    res, _ = orc.run_generated(m["np"], m["dist"], m["seed"], m["n_instr"], m["first_sys"],
                               m["n_sys"], nthreads=8)
    gold = golden_ensemble(name)
    mine = res_to_u64(res)
    bad = np.nonzero((mine != gold).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} systems differ, first {bad[:5]}"


@pytest.mark.parametrize("name", ["np8_uniform", "np8_hot", "np4_uniform"])
def test_oracle_records_match_reference_handler_text(name, ensemble_meta):
    m = ensemble_meta[name]
    tr, cn = orc.generate(m["np"], m["dist"], m["seed"], m["n_instr"], m["first_sys"], 16)
    _, _, dump, fin = orc.run_packed(m["np"], tr, cn, records=True)
    gold = golden_ensemble_recs(name)
    assert np.array_equal(dump, gold[:, 0]) and np.array_equal(fin, gold[:, 1])


def test_generator_ranges():
    for dist, ok in [("uniform", lambda a: a < 0x80), ("hot", lambda a: a in (0, 0x11, 0x22, 0x33)),
                     ("evict", lambda a: a % 4 == 0 and a < 0x80)]:
        tr, _ = orc.generate(8, dist, 3, 256, 5, 4)
        addr = (tr >> 8) & 0x7F
        assert all(ok(int(a)) for a in np.unique(addr))
        wr = tr >> 15
        assert 0.4 < wr.mean() < 0.6
        assert np.all((tr[wr == 0] & 0xFF) == 0)   # RD carries value 0 (:810)
    a, _ = orc.generate(4, "uniform", 1, 64, 0, 2)
    assert int(((a >> 8) & 0x7F).max()) < 0x40


def test_generator_is_counter_based():
    a, _ = orc.generate(8, "uniform", 1, 64, 100, 4)
    b, _ = orc.generate(8, "uniform", 1, 64, 102, 1)
    assert np.array_equal(a[2], b[0])
