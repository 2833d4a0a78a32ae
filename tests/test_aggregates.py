"""CPU: the full-size golden aggregates (tests/golden/aggregates.json).

oracle/gen_fixtures.py `aggregates` runs the reference's own handler/issue text
(oracle/_ref/ref_lockstep_np8 agg, lock-step schedule) over every system of bench.py's three
workloads -- C3 1M uniform, C4 1M hot-line, C5 2M eviction-heavy -- and of the 4096-system
golden fixtures.  bench.py compares every run's per-system results with them after the timed
region, and the full-size GPU tests do too.  Here: the numpy restatement of the per-system
result digest (pydsm.result_digest) equals the C one (dsm_common.h dsm_result_digest) on the
golden per-system fixtures, the oracle reproduces the small aggregates, and the table covers
exactly bench.py's workloads."""
import json
import os

import numpy as np
import pytest

from conftest import GOLD, REPO

import pydsm

AGG = json.load(open(os.path.join(GOLD, "aggregates.json")))


def _res(u64):
    r = np.zeros(len(u64), dtype=pydsm.RESULT_DTYPE)
    for i, k in enumerate(("status", "rounds", "msgs", "instrs")):
        r[k] = u64[:, i].astype(np.uint32)
    r["dump_hash"], r["final_hash"] = u64[:, 4], u64[:, 5]
    return r


@pytest.mark.parametrize("name", ["np8_uniform", "np8_hot", "np8_evict"])
def test_digest_matches_reference_fixture(name):
    """numpy aggregate of the reference's per-system fixture == the C aggregate of the same run."""
    g = np.load(os.path.join(GOLD, "ensemble", f"{name}.npy"))
    mine = pydsm.aggregate(_res(g))
    assert pydsm.aggregate_diff(mine, AGG[name]) == [], (mine, AGG[name])


def test_digest_is_position_sensitive():
    g = _res(np.load(os.path.join(GOLD, "ensemble", "np8_uniform.npy")))
    sw = g.copy()
    sw[[0, 1]] = sw[[1, 0]]
    assert pydsm.result_digest(sw) != pydsm.result_digest(g)
    assert pydsm.aggregate(sw)["msgs"] == pydsm.aggregate(g)["msgs"]


@pytest.mark.parametrize("name,dist", [("np8_uniform", "uniform"), ("np8_evict", "evict")])
def test_oracle_reproduces_aggregate(name, dist):
    import pyoracle
    a = AGG[name]
    res, _ = pyoracle.run_generated(8, dist, a["seed"], a["n_instr"], a["first_sys"], a["systems"],
                                    nthreads=8)
    assert pydsm.aggregate_diff(pydsm.aggregate(res), a) == []


def test_aggregates_cover_bench_configs():
    import sys
    sys.path.insert(0, REPO)
    import bench
    for cfg, (dist, n_sys, n_instr, seed, _) in bench.CONFIGS.items():
        a = AGG[cfg]
        assert (a["systems"], a["n_instr"], a["seed"], a["first_sys"], a["np"]) == \
            (n_sys, n_instr, seed, 0, bench.NP)
        assert a["dist"] == pydsm.DIST[dist]
        assert sum(a["status"]) == a["systems"]
