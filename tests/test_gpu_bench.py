"""GPU: bench.py end to end on the one GPU of the box -- the 1-rank line, `--gpus 2` through
its own launcher (both ranks on device 0, counters over gloo: RCCL needs a GPU per rank), whose
whole-job counters must equal one rank simulating both shards, the RCCL path (libdsm's
dsm_group_*: barriers, all-reduce of the counters, the aggregate and the elapsed time) at one
rank, and the C multi-GPU driver (dsm_ensemble) at one GPU."""
import json
import os
import subprocess
import sys

import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu

SMALL = ["--systems", "32768", "--steps", "2", "--warmup", "1", "--no-cpu", "--no-dump",
         "--parse-systems", "0"]


def _bench(args, env=None, timeout=240):
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, cwd=REPO,
                       capture_output=True, text=True, timeout=timeout,
                       env=dict(os.environ, **(env or {})))
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_two_rank_launch_equals_one_rank_over_both_shards():
    two = _bench(["--gpus", "2"] + SMALL,
                 env={"DSM_BENCH_BACKEND": "gloo", "DSM_BENCH_DEVICE": "0"})
    one = _bench(["--gpus", "1"] + SMALL[:1] + ["65536"] + SMALL[2:])
    assert two["n_gpus"] == 2 and one["n_gpus"] == 1
    assert two["config"]["parallelism"] == "ensemble-dp2"
    for k in ("msgs", "instrs", "rounds", "systems", "max_rounds", "status_DEADLOCKED"):
        assert two["counters"][k] == one["counters"][k], k
    assert two["sum_final_hash"] == one["sum_final_hash"]
    assert two["value"] > 0 and two["roofline"]["achieved"] > 0


def test_rccl_collective_path_one_rank():
    """bench.py's default collective path at one rank: libdsm's own RCCL communicator
    (dsm_group_init_rank over a single-rank id), the RCCL barriers around the timed region,
    the MAX all-reduce of the elapsed time and the SUM / MAX all-reduces of the counters and of
    the aggregate (dsm_group_allreduce_*) -- the same results as the run without any
    collective (the gloo backend at one rank)."""
    rccl = _bench(["--gpus", "1"] + SMALL)
    plain = _bench(["--gpus", "1"] + SMALL, env={"DSM_BENCH_BACKEND": "gloo"})
    assert rccl["collective"].startswith("rccl ncclAllReduce issued by libdsm"), rccl["collective"]
    assert plain["collective"] is None
    for k in ("msgs", "instrs", "rounds", "systems", "max_rounds", "status_DEADLOCKED"):
        assert rccl["counters"][k] == plain["counters"][k], k
    assert rccl["sum_final_hash"] == plain["sum_final_hash"]
    # the untimed per-type pass: 13 counts summing to the timed run's messages
    assert sum(rccl["msgs_by_type"].values()) == rccl["counters"]["msgs"]
    assert "msgs_by_type" in rccl["parity"] and "MISMATCH" not in rccl["parity"], rccl["parity"]


def test_c_driver_one_gpu_pinned_prefix():
    """bench.py --driver c: the C multi-GPU driver (dsm_ensemble, one host thread per GPU,
    RCCL through dsm_group_init_all) at one GPU over the 4096 systems the golden per-system
    fixture pins: its device aggregate (dsm_aggregate_device) and the reduced counters equal the
    reference's, and its per-type counts sum to the messages."""
    line = _bench(["--driver", "c", "--gpus", "1", "--systems", "4096", "--steps", "2",
                   "--warmup", "1"])
    assert line["n_gpus"] == 1 and line["driver"].startswith("dsm_ensemble (C")
    assert line["parity"].startswith("full-size aggregate == reference (job total over 1 shard(s), "
                                     "aggregates.json:np8_uniform)"), line["parity"]
    assert "1/1 shards" in line["parity"] and "MISMATCH" not in line["parity"]
    assert "msgs_by_type == reference (13 types)" in line["parity"], line["parity"]
    assert sum(line["msgs_by_type"].values()) == line["counters"]["msgs"]
    assert line["value"] > 0 and line["collective"].startswith("rccl ncclAllReduce over 1 GPU")


@pytest.mark.parametrize("gpus,config,n", [(2, "random", 2048), (4, "evict", 1024)])
def test_multi_rank_line_checks_every_shard_and_the_total(gpus, config, n):
    """`--gpus N` (every rank on device 0, gloo): each rank checks its shard's results against
    the reference's aggregate of its id range, rank 0 the all-reduced job total against the
    reference's over [0, N * n) -- the bench line's `parity` says both (here the ranges lie in
    the 4096-system golden fixtures; at full size, tests/golden/aggregates.json's <config>@<r>
    shard entries and <config>@x<N> totals)."""
    small = ["--systems", str(n)] + SMALL[2:]
    line = _bench(["--gpus", str(gpus), "--config", config] + small,
                  env={"DSM_BENCH_BACKEND": "gloo", "DSM_BENCH_DEVICE": "0"})
    assert line["n_gpus"] == gpus
    assert line["parity"].startswith(f"full-size aggregate == reference (job total over {gpus} shard(s)"), line["parity"]
    assert f"{gpus}/{gpus} shards == their reference aggregates" in line["parity"], line["parity"]
    assert line["parity_detail"]["shards"] == dict(ok=gpus, bad=0, unpinned=0)
    assert "golden[0:%d] bit-exact" % n in line["parity"]
