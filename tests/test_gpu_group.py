"""GPU: the multi-GPU reduction of the C ABI at one GPU (ABI 5) -- libdsm's own RCCL
communicator (dsm_group_*) on a single-device group, the device aggregate
(dsm_aggregate_device) against the reference's aggregates, and the C multi-GPU driver
(dsm_ensemble: one host thread per GPU, ncclCommInitAll, one ncclAllReduce of the counters and
of the aggregate) over the full C3 workload, its reduced totals and per-type message counts
against the reference's full-size aggregate (tests/golden/aggregates.json:random, from the
reference's own handler text under the lock-step schedule)."""
import json
import os
import subprocess

import numpy as np
import pytest

from conftest import PKG, golden_aggregate, golden_ensemble

import pydsm  # noqa: E402

pytestmark = pytest.mark.gpu

AGG_KEYS = ("systems", "msgs", "instrs", "rounds", "max_rounds", "status", "sum_dump_hash",
            "sum_final_hash", "result_digest")


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    if pydsm.device_count() < 1:
        pytest.fail("gpu tests need a GPU (no fallback exists)")
    return torch, torch.device("cuda", 0)


def test_single_rank_group_reductions(torch_dev):
    """A one-rank RCCL group: every all-reduce is the identity (sum and max), the mixed
    counters / aggregate reductions keep max_rounds, the barrier returns."""
    torch, dev = torch_dev
    st = torch.cuda.current_stream(dev).cuda_stream
    g = pydsm.Group(0, 1, 0, pydsm.Group.unique_id())
    try:
        assert g.info() == (0, 1, 0)
        v = torch.arange(1, 41, dtype=torch.int64, device=dev) * 977
        for op in (pydsm.RED_SUM, pydsm.RED_MAX):
            w = v.clone()
            g.allreduce(w, 40, op, st)
            torch.cuda.synchronize(dev)
            assert torch.equal(w, v)
        c = v.clone()
        g.allreduce_counters(c, st)
        a = v[:pydsm.NAGG].clone()
        g.allreduce_aggregate(a, st)
        g.barrier(st)
        assert torch.equal(c, v) and torch.equal(a, v[:pydsm.NAGG])
        with pytest.raises(pydsm.DsmError):
            g.allreduce_counters(v[:8], st)          # a buffer smaller than dsm_counters
    finally:
        g.close()


@pytest.mark.parametrize("name,first", [("np8_hot", 0), ("np8_uniform_far", 999_000)])
def test_device_aggregate_equals_reference(torch_dev, name, first):
    """dsm_aggregate_device over the reference's per-system results == the host fold and the
    reference's aggregate; a second call accumulates (sums double, the max stays)."""
    torch, dev = torch_dev
    st = torch.cuda.current_stream(dev).cuda_stream
    g = golden_ensemble(name)
    res = np.zeros(len(g), dtype=pydsm.RESULT_DTYPE)
    for i, f in enumerate(("status", "rounds", "msgs", "instrs", "dump_hash", "final_hash")):
        res[f] = g[:, i]
    d_res = torch.from_numpy(res.view(np.int64).copy()).to(dev)
    agg = torch.zeros(pydsm.NAGG, dtype=torch.int64, device=dev)
    with pydsm.Engine(8, 4096) as eng:
        eng.aggregate_device(d_res, len(res), first, agg, st)
        torch.cuda.synchronize(dev)
        one = pydsm.agg_vec_to_dict(agg.cpu().numpy().view(np.uint64))
        eng.aggregate_device(d_res, len(res), first, agg, st)
        torch.cuda.synchronize(dev)
        two = pydsm.agg_vec_to_dict(agg.cpu().numpy().view(np.uint64))
    assert one == pydsm.aggregate(res, first)
    if first == 0:
        gold = golden_aggregate(name)
        assert {k: one[k] for k in AGG_KEYS} == {k: gold[k] for k in AGG_KEYS}
    assert two["msgs"] == 2 * one["msgs"] and two["max_rounds"] == one["max_rounds"]


def test_c_driver_full_c3_equals_reference():
    """dsm_ensemble --gpus 1 over the full C3 workload (1M systems, 4096 instructions per
    node): the RCCL-reduced aggregate, counters and per-type counts == the reference's."""
    r = subprocess.run([os.path.join(PKG, "dsm_ensemble"), "--gpus", "1", "--config", "random",
                        "--steps", "1", "--warmup", "0", "--type-counts"],
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    gold = golden_aggregate("random")
    assert {k: d["total"][k] for k in AGG_KEYS} == {k: gold[k] for k in AGG_KEYS}
    assert d["ranks"][0]["aggregate"] == d["total"]
    c = d["counters"]
    assert (c["msgs"], c["instrs"], c["rounds"], c["systems"], c["max_rounds"]) == \
        (gold["msgs"], gold["instrs"], gold["rounds"], gold["systems"], gold["max_rounds"])
    assert c["sum_final_hash"] == gold["sum_final_hash"]
    assert d["msgs_by_type"] == gold["msgs_by_type"] and d["type_pass_msgs"] == gold["msgs"]
    assert d["value"] > 0 and d["collective"].startswith("rccl ncclAllReduce over 1 GPU")
