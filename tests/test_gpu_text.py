"""GPU text boundaries through the C ABI: printProcessorState (assignment.c:824-876) formatted
by fmt_kernel, byte-exact against the reference's own printProcessorState output
(tests/golden/dumps md5s), the lock-step golden dumps, and the host formatter."""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLD, TESTS, golden_dump, inputs_dir

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dsm():
    import pydsm
    if pydsm.device_count() < 1:
        pytest.fail("gpu tests need a GPU (no fallback exists)")
    return pydsm


@pytest.fixture(scope="module")
def torch():
    import torch
    return torch


def _md5(b):
    return hashlib.md5(b).hexdigest()


def _format_on_gpu(dsm, torch, eng, recs, stride=1):
    """recs: uint8 [n, 64] host array -> (texts as bytes list, lengths)"""
    n = recs.shape[0] // stride
    d_rec = torch.from_numpy(np.ascontiguousarray(recs)).cuda()
    d_txt = torch.full((max(n, 1) * dsm.DUMP_SLOT,), 0xAB, dtype=torch.uint8, device="cuda")
    d_len = torch.zeros(max(n, 1), dtype=torch.int32, device="cuda")
    eng.format_dumps_device(d_rec.data_ptr(), n, d_txt.data_ptr(), d_len.data_ptr(), stride,
                            torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    txt = d_txt.cpu().numpy().reshape(-1, dsm.DUMP_SLOT)[:n]
    lens = d_len.cpu().numpy()[:n]
    return txt, lens


def test_gpu_format_matches_reference_printProcessorState(dsm, torch):
    recs = np.load(os.path.join(GOLD, "dumps", "random_recs.npy"))
    with open(os.path.join(GOLD, "dumps", "random_md5.json")) as f:
        texts = json.load(f)["texts"]
    with dsm.Engine(8, 8) as eng:
        txt, lens = _format_on_gpu(dsm, torch, eng, recs)
    for k in range(len(recs)):
        n = int(lens[k])
        assert n == texts[k]["len"], k
        assert _md5(bytes(txt[k, :n])) == texts[k]["md5"], k
        assert not txt[k, n:].any(), k          # slot tail is zero


@pytest.mark.parametrize("np_", [4, 8])
def test_gpu_format_odd_counts_strides_and_invalid_states(dsm, torch, np_):
    """ragged record counts (not a multiple of the 16-record workgroup tile), a record stride
    of 2 (the engine's [dump, final] layout) and out-of-range enum values, whose text follows
    the host helper's "??" / "????" convention (the reference would index out of bounds)."""
    rng = np.random.default_rng(np_)
    for n in (1, 15, 17, 1000):
        recs = rng.integers(0, 256, (2 * n, 64), dtype=np.uint8)
        with dsm.Engine(np_, 8) as eng:
            txt, lens = _format_on_gpu(dsm, torch, eng, recs, stride=2)
        for k in range(n):
            ref = dsm.format_dump(k % np_, recs[2 * k]).encode()
            assert bytes(txt[k, :lens[k]]) == ref, (n, k)


@pytest.mark.parametrize("test", TESTS)
def test_gpu_format_run_dumps_shipped_tests(dsm, torch, test):
    import pyoracle as orc
    tr, cn = orc.load_test(inputs_dir(test))
    with dsm.Engine(4, 32, snapshots=True) as eng:
        res, _ = eng.run_packed(tr, cn)
        d_txt = torch.zeros(4 * dsm.DUMP_SLOT, dtype=torch.uint8, device="cuda")
        d_len = torch.zeros(4, dtype=torch.int32, device="cuda")
        eng.format_run_dumps_device(dsm.VIEW_DUMP, 0, 1, d_txt.data_ptr(), d_len.data_ptr(),
                                    torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        texts = dsm.split_dumps(d_txt.cpu().numpy(), d_len.cpu().numpy())
    dumped = int(res[0]["status"]) >> 8
    for core in range(4):
        g = golden_dump(test, core)
        assert ((dumped >> core) & 1) == (g is not None)
        if g is not None:
            assert texts[core] == g


def test_write_run_dumps_files(dsm, tmp_path):
    import pyoracle as orc
    tr, cn = orc.load_test(inputs_dir("test_1"))
    with dsm.Engine(4, 32, snapshots=True) as eng:
        res, _ = eng.run_packed(tr, cn)
        eng.write_run_dumps(0, int(res[0]["status"]) >> 8, str(tmp_path))
    for core in range(4):
        assert (tmp_path / f"core_{core}_output.txt").read_text() == golden_dump("test_1", core)


def test_gpu_format_full_size_final_view(dsm, torch):
    """C3 at full size (1M 8-node systems): the final record of every node formatted in one
    launch; lengths follow the EXCLUSIVE count, a sample of texts equals the host formatter."""
    n_sys = 1 << 20
    dev = torch.device("cuda")
    st = torch.cuda.current_stream().cuda_stream
    with dsm.Engine(8, 4096, snapshots=True) as eng:
        out = torch.empty((n_sys, 4), dtype=torch.int64, device=dev)
        cnt = torch.zeros(32, dtype=torch.int64, device=dev)
        eng.run_generated_device("uniform", 1, 4096, 0, n_sys, out.data_ptr(), cnt.data_ptr(), st)
        d_txt = torch.empty(n_sys * 8 * dsm.DUMP_SLOT, dtype=torch.uint8, device=dev)
        d_len = torch.zeros(n_sys * 8, dtype=torch.int32, device=dev)
        eng.format_run_dumps_device(dsm.VIEW_FINAL, 0, n_sys, d_txt.data_ptr(), d_len.data_ptr(), st)
        torch.cuda.synchronize()
        lens = d_len.cpu().numpy()
        rng = np.random.default_rng(7)
        pick = np.sort(rng.choice(n_sys * 8, 2000, replace=False))
        txt = d_txt.view(-1, dsm.DUMP_SLOT)[torch.from_numpy(pick).to(dev)].cpu().numpy()
        recs = [eng.node_state(int(k) // 8, int(k) % 8)[1] for k in pick]
    assert lens.min() >= dsm.DUMP_BASE and lens.max() <= dsm.DUMP_MAX
    for i, k in enumerate(pick):
        assert bytes(txt[i, :lens[k]]) == dsm.format_dump(int(k) % 8, recs[i]).encode(), k
        assert lens[k] == dsm.DUMP_BASE + int((recs[i][56:60] == 1).sum())
    del d_txt
