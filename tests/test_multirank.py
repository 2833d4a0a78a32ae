"""N>1 path of bench.py on CPU: world_size-2 gloo process group.  Each rank simulates its
shard of system ids (bench.shard: weak scaling, contiguous ids, counter-based generator) and
the counters are combined with bench.reduce_counters (sum mod 2^64, max for max_rounds).
The compute step here is the CPU oracle, injected by the test (no GPU in this container);
the point is that sharding + reduction reproduce the single-process totals exactly."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import REPO

import pydsm  # noqa: E402  (numpy + ctypes only; the library loads lazily)

N_PER_RANK = 96


def counters_from_results(res):
    """dsm_counters layout (include/dsm.h) from per-system results."""
    c = np.zeros(pydsm.NCOUNTERS, dtype=np.uint64)
    c[13] = res["msgs"].sum(dtype=np.uint64)
    c[14] = res["instrs"].sum(dtype=np.uint64)
    c[15] = res["rounds"].sum(dtype=np.uint64)
    c[16] = len(res)
    for st in range(5):
        c[17 + st] = np.sum((res["status"] & 0xFF) == st)
    c[22] = res["dump_hash"].sum(dtype=np.uint64)
    c[23] = res["final_hash"].sum(dtype=np.uint64)
    c[24] = res["rounds"].max() if len(res) else 0
    return c


def _worker(rank, world, port, out_path):
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    import bench
    import pyoracle
    dist.init_process_group("gloo", rank=rank, world_size=world)
    first, n = bench.shard(rank, N_PER_RANK)
    res, _ = pyoracle.run_generated(8, "uniform", 1, 4096, first, n, nthreads=1)
    vec = torch.from_numpy(counters_from_results(res).view(np.int64).copy())
    tot = bench.reduce_counters(vec, dist)
    if rank == 0:
        np.save(out_path, tot.numpy().view(np.uint64))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_rank_shard_and_reduce(tmp_path):
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import pyoracle
    out = str(tmp_path / "tot.npy")
    mp.start_processes(_worker, args=(2, _free_port(), out), nprocs=2, join=True,
                       start_method="spawn")
    tot = np.load(out)
    res, _ = pyoracle.run_generated(8, "uniform", 1, 4096, 0, 2 * N_PER_RANK, nthreads=1)
    ref = counters_from_results(res)
    assert np.array_equal(tot, ref)
    assert int(tot[16]) == 2 * N_PER_RANK


def test_shard_is_contiguous_and_disjoint():
    sys.path.insert(0, REPO)
    import bench
    spans = [bench.shard(r, 1000) for r in range(8)]
    assert spans[0] == (0, 1000)
    for (a, n), (b, _) in zip(spans, spans[1:]):
        assert a + n == b


def test_results_do_not_depend_on_sharding():
    """Counter-based generator: a system's result depends only on its id."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import pyoracle
    whole, _ = pyoracle.run_generated(8, "hot", 3, 4096, 0, 64, nthreads=1)
    a, _ = pyoracle.run_generated(8, "hot", 3, 4096, 0, 40, nthreads=1)
    b, _ = pyoracle.run_generated(8, "hot", 3, 4096, 40, 24, nthreads=1)
    assert whole.tobytes() == np.concatenate([a, b]).tobytes()


def _res_from_fixture(name, lo, n):
    import pydsm
    g = np.load(os.path.join(REPO, "tests", "golden", "ensemble", f"{name}.npy"))[lo:lo + n]
    r = np.zeros(n, dtype=pydsm.RESULT_DTYPE)
    for i, k in enumerate(("status", "rounds", "msgs", "instrs", "dump_hash", "final_hash")):
        r[k] = g[:, i]
    return r


def _parity_worker(rank, world, port, n, corrupt_rank, out_path):
    """bench.py's parity path at world_size `world` over gloo: each rank checks its shard of
    the golden per-system fixture (standing in for the GPU's results), the aggregate vectors
    are all-reduced, rank 0 checks the job total."""
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "hp-assignment-2_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    import bench
    import pydsm
    dist.init_process_group("gloo", rank=rank, world_size=world)
    first, nn = bench.shard(rank, n)
    res = _res_from_fixture("np8_uniform", first, nn)
    if rank == corrupt_rank:
        res["final_hash"][nn // 2] ^= np.uint64(1)
    cvec = torch.from_numpy(counters_from_results(res).view(np.int64).copy())
    tot = bench.reduce_counters(cvec, dist)
    c = pydsm.counters_to_dict(tot.numpy().view(np.uint64))
    local_c = pydsm.counters_to_dict(counters_from_results(res))
    mine, verdict, msg = bench.shard_parity("uniform", 1, 4096, first, res, local_c)
    avec = torch.from_numpy(bench.agg_to_vec(mine, verdict).view(np.int64).copy())
    avec = bench.reduce_vector(avec, dist, (bench.AGG_MAX,))
    parity, detail = bench.job_parity("uniform", 1, 4096, world, n, avec.numpy().view(np.uint64), c)
    with open(f"{out_path}.{rank}", "w") as f:
        f.write(f"{verdict}\n{msg}\n{parity}\n")
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,corrupt", [(2, -1), (4, -1), (2, 1)])
def test_bench_parity_every_shard_and_job_total(tmp_path, world, corrupt):
    """Every rank checks its shard against the reference aggregate of its id range and rank 0
    the all-reduced job total against the reference's total over [0, world * n): the same
    functions bench.py runs after its timed region (4096-system golden fixture, gloo)."""
    out = str(tmp_path / "p")
    n = 4096 // world
    mp.start_processes(_parity_worker, args=(world, _free_port(), n, corrupt, out), nprocs=world,
                       join=True, start_method="spawn")
    lines = [open(f"{out}.{r}").read().splitlines() for r in range(world)]
    for r, (verdict, msg, _) in enumerate(lines):
        assert verdict == ("bad" if r == corrupt else "ok"), msg
        assert msg.startswith(f"shard [{r * n}, {(r + 1) * n})")
    parity = lines[0][2]
    if corrupt < 0:
        assert parity.startswith(f"full-size aggregate == reference (job total over {world} shard(s), "
                                 "aggregates.json:np8_uniform)"), parity
        assert parity.endswith(f"{world}/{world} shards == their reference aggregates"), parity
    else:
        assert parity.startswith("AGGREGATE MISMATCH vs aggregates.json:np8_uniform"), parity
        assert "1 SHARD MISMATCH" in parity
