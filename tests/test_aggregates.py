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


# -- multi-GPU bench: per-shard reference aggregates and the 2/4/8-GPU job totals
#    (oracle/gen_fixtures.py shards; bench.golden_for / shard_parity / job_parity)

def _bench():
    import sys
    sys.path.insert(0, REPO)
    import bench
    return bench


def _gen():
    import gen_fixtures
    return gen_fixtures


def test_merge_of_ranges_equals_one_range():
    """The identity the job totals rest on: the aggregate of [0, n) is the merge of the
    aggregates of a split of it (sums mod 2^64 of the hashes and the position-sensitive
    digest, max of max_rounds)."""
    g = _res(np.load(os.path.join(GOLD, "ensemble", "np8_uniform.npy")))
    whole = pydsm.aggregate(g)
    for cut in (1, 1000, 2048, 4095):
        parts = [pydsm.aggregate(g[:cut], 0), pydsm.aggregate(g[cut:], cut)]
        assert pydsm.aggregate_diff(_gen().merge_aggregates(parts), whole) == []
    # the digest pins positions: the same slice at the wrong offset differs
    assert pydsm.aggregate(g[1000:], 0)["result_digest"] != pydsm.aggregate(g[1000:], 1000)["result_digest"]


def test_reference_run_equals_merge_of_its_slices():
    """One reference run over ids [0, 3000) == the merge of runs over [0, 1000) and
    [1000, 3000): the check behind the "<config>@x<N>" totals (skipped without oracle/_ref)."""
    import subprocess
    exe = os.path.join(REPO, "oracle", "_ref", "ref_lockstep_np8")
    if not os.path.exists(exe):
        pytest.skip("oracle/_ref not built")

    def agg(first, n):
        r = subprocess.run([exe, "agg", "2", "1", "4096", str(first), str(n), "4"], check=True,
                           capture_output=True, text=True)
        return json.loads(r.stdout.strip().splitlines()[-1])
    whole = agg(0, 3000)
    assert pydsm.aggregate_diff(_gen().merge_aggregates([agg(0, 1000), agg(1000, 2000)]), whole) == []


SHARDED = [k for k in ("random", "hot", "evict") if f"{k}@x8" in AGG]


@pytest.mark.parametrize("cfg", SHARDED)
def test_shard_entries_and_job_totals(cfg):
    """Shards 1..7 of every bench workload hold the reference's aggregate of ids
    [r*n, (r+1)*n), and the 2/4/8-GPU totals are the merge of shards 0..N-1."""
    base = AGG[cfg]
    n = base["systems"]
    parts = [base] + [AGG[f"{cfg}@{r}"] for r in range(1, 8)]
    for r, p in enumerate(parts):
        assert (p["first_sys"], p["systems"], p["dist"], p["seed"], p["n_instr"]) == \
            (r * n, n, base["dist"], base["seed"], base["n_instr"])
        assert sum(p["status"]) == n
    assert len({p["result_digest"] for p in parts}) == 8
    for g in (2, 4, 8):
        t = AGG[f"{cfg}@x{g}"]
        assert t["systems"] == g * n and t["first_sys"] == 0
        assert pydsm.aggregate_diff(_gen().merge_aggregates(parts[:g]), t) == []


def test_all_bench_shards_are_pinned():
    """Every rank of a 1/2/4/8-GPU bench run finds its shard's reference aggregate, and rank 0
    the job total (bench.golden_for), for every workload whose shards are generated."""
    bench = _bench()
    for cfg in SHARDED:
        dname, n, n_instr, seed, _ = bench.CONFIGS[cfg]
        for world in (1, 2, 4, 8):
            for r in range(world):
                first, nn = bench.shard(r, n)
                g, src = bench.golden_for(dname, seed, n_instr, first, nn)
                assert g is not None and src.startswith("aggregates.json:"), (cfg, world, r)
            g, src = bench.golden_for(dname, seed, n_instr, 0, world * n)
            assert src == "aggregates.json:" + (cfg if world == 1 else f"{cfg}@x{world}")


def test_golden_for_small_ranges_come_from_fixtures():
    bench = _bench()
    g, src = bench.golden_for("uniform", 1, 4096, 2048, 1024)
    assert src == "ensemble/np8_uniform.npy[2048:3072]"
    fx = _res(np.load(os.path.join(GOLD, "ensemble", "np8_uniform.npy")))
    assert pydsm.aggregate_diff(pydsm.aggregate(fx[2048:3072], 2048), g) == []
    g, src = bench.golden_for("uniform", 1, 4096, 999_100, 100)
    assert src == "ensemble/np8_uniform_far.npy[100:200]"
    assert bench.golden_for("uniform", 1, 4096, 4000, 200) == (None, None)
    assert bench.golden_for("hot", 2, 4096, 0, 16) == (None, None)
