"""GPU: bench.py end to end on the one GPU of the box -- the 1-rank line, `--gpus 2` through
its own launcher (both ranks on device 0, counters over gloo: RCCL needs a GPU per rank), whose
whole-job counters must equal one rank simulating both shards, and the RCCL path (process
group, barriers, all-reduce of the counters and of the elapsed time) at one rank."""
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
    """bench.py's torch.distributed path on the nccl backend (RCCL), forced at world size 1:
    init with device_id, the barriers around the timed region, the MAX all-reduce of the
    elapsed time and the SUM / MAX all-reduce of the counters -- the same results as the plain
    run."""
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    env = {"RANK": "0", "LOCAL_RANK": "0", "WORLD_SIZE": "1", "LOCAL_WORLD_SIZE": "1",
           "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "DSM_BENCH_DIST": "1"}
    rccl = _bench(["--gpus", "1"] + SMALL, env=env)
    plain = _bench(["--gpus", "1"] + SMALL)
    assert rccl["collective"].startswith("rccl all_reduce") and plain["collective"] is None
    for k in ("msgs", "instrs", "rounds", "systems", "max_rounds", "status_DEADLOCKED"):
        assert rccl["counters"][k] == plain["counters"][k], k
    assert rccl["sum_final_hash"] == plain["sum_final_hash"]


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
