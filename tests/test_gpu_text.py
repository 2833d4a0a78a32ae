"""GPU text boundaries through the C ABI: printProcessorState (assignment.c:824-876) formatted
by fmt_kernel, byte-exact against the reference's own printProcessorState output
(tests/golden/dumps md5s), the lock-step golden dumps, and the host formatter."""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLD, TESTS, golden_dump, inputs_dir

import pydsm  # noqa: E402  (numpy + ctypes only; the library loads lazily)

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
        cnt = torch.zeros(pydsm.NCOUNTERS, dtype=torch.int64, device=dev)
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


# ---- initializeProcessor's reader on the GPU (parse_kernel) --------------------------------
def _host_expect(dsm, tmp_path, files, np_, cap):
    """Expected (count, status, traces) per file from the host reader dsm_parse_trace_file
    (glibc fgets + sscanf, the reference's :802-818 recipe) plus the home < np check."""
    import ctypes
    out = []
    p = tmp_path / "core.txt"
    for data in files:
        p.write_bytes(data)
        buf = np.zeros(max(cap, 1), dtype=np.uint16)
        n = ctypes.c_uint32(0)
        rc = dsm.lib().dsm_parse_trace_file(str(p).encode(), ctypes.c_void_p(buf.ctypes.data), cap,
                                            ctypes.byref(n))
        n = n.value
        bad = np.nonzero(((buf[:n] >> 12) & 7) >= np_)[0]
        if bad.size:
            n, rc = int(bad[0]), dsm.E_RANGE
        out.append((n, rc, buf[:n].copy()))
    return out


LINES = [b"RD 0x00\n", b"RD 0x1f\n", b"WR 0x02 100\n", b"WR 0x3f 255\n", b"WR 0x10 300\n",
         b"RD 0x7f\n", b"WR 0x45 -1\n", b"RD 1F\n", b"RD\t0X2a\n", b"WR 0x11   +7\n",
         b"RD 0x01\r\n", b"WR 0x00 0\n", b"RD 0x0\n", b"RD 0x\n", b"WR 0x2 08\n",
         b"RD 0x11          RD 0x05\n",              # long line: second chunk is its own RD
         b"WR 0x12 1                 \n",            # long line: the tail chunk is FORMAT
         b"RD 0x13" + b" " * 12 + b"\n",             # 19 chars + '\n': the '\n' alone is a chunk
         b"\n", b"XX 0x1\n", b"RD zz\n", b"WR 0x05\n", b"RD 0x80\n"]


def _fuzz_files(rng, n_files, max_lines, bad_rate):
    good = LINES[:15]
    files = []
    for _ in range(n_files):
        k = int(rng.integers(0, max_lines + 1))
        pick = [good[i] for i in rng.integers(0, len(good), k)]
        if k and rng.random() < bad_rate:
            pick[int(rng.integers(0, k))] = LINES[int(rng.integers(15, len(LINES)))]
        data = b"".join(pick)
        if data and rng.random() < 0.2:
            data = data[:-1]                         # no trailing newline
        files.append(data)
    return files


@pytest.mark.parametrize("np_,cap", [(4, 32), (8, 32), (8, 4096)])
def test_gpu_parse_fuzzed_files_equal_host_reader(dsm, tmp_path, np_, cap):
    rng = np.random.default_rng(cap + np_)
    files = _fuzz_files(rng, 64 * np_, 60 if cap == 32 else 300, 0.3)
    exp = _host_expect(dsm, tmp_path, files, np_, cap)
    with dsm.Engine(np_, cap) as eng:
        tr, cn, st = eng.parse_traces(files, cap)
    tr, cn, st = tr.reshape(len(files), -1), cn.reshape(-1), st.reshape(-1)
    for f, (n, rc, t) in enumerate(exp):
        assert (int(cn[f]), int(st[f])) == (n, rc), (f, files[f][:200])
        assert np.array_equal(tr[f, :n], t), f


def test_gpu_parse_shipped_tests_and_cli_inputs(dsm):
    import pyoracle as orc
    files, exp = [], []
    for test in TESTS:
        for core in range(4):
            files.append(open(os.path.join(inputs_dir(test), f"core_{core}.txt"), "rb").read())
        exp.append(orc.load_test(inputs_dir(test)))
    with dsm.Engine(4, 32) as eng:
        tr, cn, st = eng.parse_traces(files, 32)
    assert not st.any()
    for i, (etr, ecn) in enumerate(exp):
        assert np.array_equal(cn[i], ecn[0])
        for core in range(4):
            assert np.array_equal(tr[i, core, :cn[i, core]], etr[0, core, :ecn[0, core]])


def test_gpu_parse_window_edges(dsm, tmp_path):
    """files whose lines straddle the 1 KB window and 16-byte lane boundaries, long runs of
    blank-free text, offsets that are not 16-byte aligned, and empty files."""
    files = []
    for pad in range(0, 40):
        body = b"".join(LINES[i % 15] for i in range(pad, pad + 400))
        files.append(b"RD 0x01" + b" " * (pad % 12) + b"\n" + body)
    files += [b"", b"RD 0x01", b"WR 0x10 5"]
    while len(files) % 4:
        files.append(b"")
    exp = _host_expect(dsm, tmp_path, files, 4, 512)
    with dsm.Engine(4, 512) as eng:
        tr, cn, st = eng.parse_traces(files, 512)
    tr, cn, st = tr.reshape(len(files), -1), cn.reshape(-1), st.reshape(-1)
    for f, (n, rc, t) in enumerate(exp):
        assert (int(cn[f]), int(st[f])) == (n, rc), f
        assert np.array_equal(tr[f, :n], t), f


@pytest.mark.parametrize("dist", ["uniform", "hot", "evict"])
def test_gpu_text_generator_round_trip(dsm, torch, dist):
    """synthetic text files (generator -> text on the GPU) parse back to exactly the packed
    traces of gen_kernel; a sample of files is also checked with the host reader."""
    n_sys, n_instr = 2048, 4096
    st = torch.cuda.current_stream().cuda_stream
    with dsm.Engine(8, n_instr) as eng:
        off = torch.zeros(n_sys * 8 + 1, dtype=torch.int64, device="cuda")
        eng.generate_text_device(dist, 1, n_instr, 5000, n_sys, 0, off.data_ptr(), st)
        torch.cuda.synchronize()
        total = int(off[-1].item())
        txt = torch.zeros(total + 64, dtype=torch.uint8, device="cuda")
        eng.generate_text_device(dist, 1, n_instr, 5000, n_sys, txt.data_ptr(), off.data_ptr(), st)
        tr = torch.zeros((n_sys, 8, n_instr), dtype=torch.int16, device="cuda")
        cn = torch.zeros((n_sys, 8), dtype=torch.int32, device="cuda")
        ss = torch.full((n_sys, 8), 99, dtype=torch.int32, device="cuda")
        eng.parse_traces_device(txt.data_ptr(), off.data_ptr(), n_sys * 8, n_instr, tr.data_ptr(),
                                cn.data_ptr(), ss.data_ptr(), st)
        gtr = torch.zeros_like(tr)
        gcn = torch.zeros_like(cn)
        eng.generate_device(dist, 1, n_instr, 5000, n_sys, gtr.data_ptr(), gcn.data_ptr(), st)
        torch.cuda.synchronize()
        assert int(ss.abs().sum().item()) == 0
        assert torch.equal(cn, gcn) and torch.equal(tr, gtr)
        o = off.cpu().numpy()
        t = txt.cpu().numpy()
        files = [bytes(t[o[f]:o[f + 1]]) for f in (0, 1, 777, n_sys * 8 - 1)]
        assert all(fl.startswith((b"RD 0x", b"WR 0x")) and fl.endswith(b"\n") for fl in files)


# valid lines longer than fgets' 19 bytes: each 19-byte chunk is a whole instruction
LONG_OK = [b"RD 0x11" + b" " * 12 + b"RD 0x05\n",
           b"WR 0x12 100" + b" " * 8 + b"WR 0x3f 7\n",
           b"RD 0x01" + b" " * 12 + b"RD 0x02" + b" " * 12 + b"RD 0x03\n"]


@pytest.mark.gpu
@pytest.mark.parametrize("rate", [0.0005, 0.01, 0.2])
def test_gpu_parse_sparse_long_lines_equal_host_reader(dsm, tmp_path, rate):
    """Multi-window files whose valid long lines come at random, sparse to dense: windows with
    and without a long line alternate, so both the line-start shortcut and the exact chunk
    numbering (parse_kernel, :802-818 fgets(line, 20)) run and hand over line starts."""
    rng = np.random.default_rng(int(rate * 1e4))
    good = LINES[:6]
    files = []
    for _ in range(48):
        k = int(rng.integers(200, 1500))
        pick = [LONG_OK[int(rng.integers(0, 3))] if rng.random() < rate else good[int(rng.integers(0, 6))]
                for _ in range(k)]
        files.append(b"".join(pick))
    cap = 4096
    exp = _host_expect(dsm, tmp_path, files, 8, cap)
    with dsm.Engine(8, cap) as eng:
        tr, cn, st = eng.parse_traces(files, cap)
    tr, cn, st = tr.reshape(len(files), -1), cn.reshape(-1), st.reshape(-1)
    for f, (n, rc, t) in enumerate(exp):
        assert (int(cn[f]), int(st[f])) == (n, rc), f
        assert np.array_equal(tr[f, :n], t), f
