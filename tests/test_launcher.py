"""bench.py's rank launcher (no GPU): `python bench.py --gpus N` without a torch.distributed
launcher starts N fresh rank processes with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR /
MASTER_PORT set, relays rank 0's output and fails when a rank fails."""
import json
import os
import sys

from conftest import REPO

sys.path.insert(0, REPO)
import bench  # noqa: E402

ECHO = ("import json, os, sys; d = {k: os.environ.get(k) for k in "
        "('RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'LOCAL_WORLD_SIZE', 'MASTER_ADDR', 'MASTER_PORT')};"
        "d['argv'] = sys.argv[1:];"
        "open(os.path.join(sys.argv[1], 'rank%s.json' % d['RANK']), 'w').write(json.dumps(d))")


def test_spawns_n_ranks_with_env(tmp_path):
    rc = bench.launch_ranks(4, [str(tmp_path), "--gpus", "4"], cmd=[sys.executable, "-c", ECHO],
                            timeout=120)
    assert rc == 0
    ds = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(4)]
    for r, d in enumerate(ds):
        assert d["RANK"] == d["LOCAL_RANK"] == str(r)
        assert d["WORLD_SIZE"] == d["LOCAL_WORLD_SIZE"] == "4"
        assert d["MASTER_ADDR"] == "127.0.0.1"
        assert d["argv"] == [str(tmp_path), "--gpus", "4"]
    assert len({d["MASTER_PORT"] for d in ds}) == 1


def test_failing_rank_fails_the_launch(tmp_path):
    # rank 1 fails at once; rank 0 would otherwise wait for it (as in a barrier)
    code = ("import os, sys, time\n"
            "if os.environ['RANK'] == '1': sys.exit(3)\n"
            "time.sleep(60)\n")
    rc = bench.launch_ranks(2, [], cmd=[sys.executable, "-c", code], timeout=120)
    assert rc == 3


def test_rank0_output_is_relayed(tmp_path, capfd):
    code = "import os; print('{\"rank\": %s}' % os.environ['RANK']) if os.environ['RANK'] == '0' else print('noise')"
    assert bench.launch_ranks(3, [], cmd=[sys.executable, "-c", code], timeout=120) == 0
    out = capfd.readouterr().out.strip().splitlines()
    assert out == ['{"rank": 0}']


def test_host_cpu_description():
    hc = bench.host_cpu()
    assert hc["threads"] >= 1 and hc["nproc"] >= hc["affinity"] >= 1
    assert isinstance(hc["model"], str)


def test_host_cpu_respects_the_job_share(monkeypatch):
    """The CPU baselines run on the job's CPU share: OMP_NUM_THREADS (the pool sets it to the
    share) caps the workers, never above the CPUs this process may run on; the report keeps
    the whole machine's nproc next to it (for the full-host estimate)."""
    monkeypatch.setenv("OMP_NUM_THREADS", "3")
    hc = bench.host_cpu()
    assert 1 <= hc["threads"] <= 3 and hc["threads"] <= hc["affinity"]
    assert hc["nproc"] == os.cpu_count() and hc["omp_num_threads"] == "3"
    monkeypatch.delenv("OMP_NUM_THREADS")
    hc = bench.host_cpu()
    assert hc["threads"] <= hc["affinity"] and hc["omp_num_threads"] is None
    q = bench.cgroup_cpus()
    if q is not None:
        assert hc["threads"] <= max(1, int(q))
