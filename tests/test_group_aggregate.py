"""CPU: the per-system aggregate of the C ABI (ABI 5: dsm_aggregate_results, dsm_result_digest)
against the reference's golden aggregates, and the layout contracts the multi-GPU all-reduce
relies on (dsm_aggregate = DSM_NAGG uint64 with max_rounds at DSM_AGG_MAX_SLOT; the C driver
and bench.py reduce it as one vector).  No GPU: host functions of libdsm.so only."""
import json
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import GOLD, PKG, REPO, golden_aggregate, golden_ensemble

import pydsm  # noqa: E402


def _results(name):
    g = golden_ensemble(name)
    res = np.zeros(len(g), dtype=pydsm.RESULT_DTYPE)
    for i, f in enumerate(("status", "rounds", "msgs", "instrs", "dump_hash", "final_hash")):
        res[f] = g[:, i]
    return res


AGG_KEYS = ("systems", "msgs", "instrs", "rounds", "max_rounds", "status", "sum_dump_hash",
            "sum_final_hash", "result_digest")


@pytest.mark.parametrize("name", ["np8_uniform", "np8_hot", "np8_evict"])
def test_host_aggregate_equals_reference(name):
    """dsm_aggregate_results over the reference's per-system results of a golden ensemble ==
    the reference's own aggregate of the same systems (ref_lockstep agg)."""
    res = _results(name)
    mine = pydsm.aggregate_results_c(res, 0)
    gold = golden_aggregate(name)
    assert {k: mine[k] for k in AGG_KEYS} == {k: gold[k] for k in AGG_KEYS}
    assert mine == pydsm.aggregate(res, 0)


def test_aggregate_merges_by_shard():
    """Shards of an ensemble merge by addition (and a max): the position-sensitive digest
    uses absolute ids, so [0, n) == [0, k) + [k, n) for every split."""
    res = _results("np8_uniform")
    whole = int(pydsm.aggregate_results_c(res, 0)["result_digest"], 16)
    for k in (1, 1000, 2048, 4095):
        a, b = pydsm.aggregate_results_c(res[:k], 0), pydsm.aggregate_results_c(res[k:], k)
        dig = (int(a["result_digest"], 16) + int(b["result_digest"], 16)) & ((1 << 64) - 1)
        assert dig == whole
        assert a["msgs"] + b["msgs"] == sum(int(x) for x in res["msgs"])
        assert max(a["max_rounds"], b["max_rounds"]) == int(res["rounds"].max())


def test_result_digest_per_system():
    """dsm_result_digest(id, r) summed over systems == the aggregate's result_digest."""
    import ctypes
    res = _results("np8_evict")[:64]
    L = pydsm.lib()
    tot = 0
    for i in range(len(res)):
        r = np.ascontiguousarray(res[i:i + 1])
        tot = (tot + L.dsm_result_digest(i + 500, ctypes.c_void_p(r.ctypes.data))) & ((1 << 64) - 1)
    assert tot == int(pydsm.aggregate_results_c(res, 500)["result_digest"], 16)


def test_aggregate_layout_and_group_symbols():
    """The header's dsm_aggregate is DSM_NAGG uint64 with max_rounds at DSM_AGG_MAX_SLOT (the
    slot the all-reduce takes a max of), pydsm mirrors it, and libdsm.so exports the group
    entry points (linked against RCCL)."""
    hdr = open(os.path.join(REPO, "include", "dsm.h")).read()
    assert re.search(r"#define DSM_NAGG\s+16\b", hdr) and re.search(r"#define DSM_AGG_MAX_SLOT\s+4\b", hdr)
    body = re.search(r"typedef struct dsm_aggregate \{(.*?)\} dsm_aggregate;", hdr, re.S).group(1)
    names = []
    for m in re.finditer(r"uint64_t\s+(\w+)(?:\[(\d+)\])?;", body):
        names += [m.group(1)] if not m.group(2) else [f"{m.group(1)}{i}" for i in range(int(m.group(2)))]
    assert len(names) == pydsm.NAGG and names[4] == "max_rounds"
    assert pydsm.AGG_FIELDS[4] == "max_rounds"
    out = subprocess.run(["nm", "-D", os.path.join(PKG, "libdsm.so")], capture_output=True,
                         text=True, check=True).stdout
    for f in ("dsm_group_unique_id", "dsm_group_init_rank", "dsm_group_init_all",
              "dsm_group_allreduce", "dsm_group_allreduce_counters",
              "dsm_group_allreduce_aggregate", "dsm_group_barrier", "dsm_group_close",
              "dsm_aggregate_device", "dsm_aggregate_results", "dsm_result_digest"):
        assert re.search(r" T %s$" % f, out, re.M), f
    ldd = subprocess.run(["readelf", "-d", os.path.join(PKG, "libdsm.so")], capture_output=True,
                         text=True, check=True).stdout
    assert "librccl.so" in ldd


def test_reference_type_totals_are_consistent():
    """Every reference aggregate carries the handled messages per transactionType
    (assignment.c:20-34; oracle/gen_fixtures.py types): they sum to its messages, and the
    2/4/8-GPU job totals are the sums of their shards'."""
    agg = json.load(open(os.path.join(GOLD, "aggregates.json")))
    for k, d in agg.items():
        assert len(d["msgs_by_type"]) == 13 and sum(d["msgs_by_type"]) == d["msgs"], k
    for cfg in ("random", "hot", "evict"):
        for g in (2, 4, 8):
            shards = [agg[cfg]] + [agg[f"{cfg}@{r}"] for r in range(1, g)]
            assert agg[f"{cfg}@x{g}"]["msgs_by_type"] == [sum(x) for x in zip(*(s["msgs_by_type"] for s in shards))]


def test_ensemble_driver_usage_without_gpu():
    """The C multi-GPU driver is built and refuses to run without a gfx950 (no CPU fallback)."""
    exe = os.path.join(PKG, "dsm_ensemble")
    assert os.access(exe, os.X_OK)
    r = subprocess.run([exe, "--bogus"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "usage" in r.stderr
