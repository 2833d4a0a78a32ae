"""GPU: the statuses of the defined deviations, produced on the device and
compared with the oracle (and, where built, the reference's own handler text):

  ASSERT_FAILED  -- an instruction whose home node is >= np (device traces are not validated;
                    the reference would index out of bounds, assignment.c:90, :602-604);
  ROUND_LIMIT    -- dsm_set_round_limit (tests/test_gpu_fastforward.py covers it inside
                    hit runs; here on message-bound systems);
  RING_OVERFLOW  -- an inbox append beyond dsm_set_inbox_limit (MSG_BUFFER_SIZE, :12; the
                    reference spins at :715-724), through the fast kernel's hand-off to the
                    256-deep re-run;
and the clamping of device trace counts above max_instr."""
import os
import subprocess
import tempfile

import numpy as np
import pytest

from conftest import ORACLE, res_to_u64

import pydsm  # noqa: E402  (numpy + ctypes only; the library loads lazily)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dsm():
    import pydsm
    if pydsm.device_count() < 1:
        pytest.fail("gpu tests need a GPU (no fallback exists)")
    return pydsm


@pytest.fixture(scope="module")
def orc():
    import pyoracle
    return pyoracle


def _cmp(a, b):
    a, b = res_to_u64(a), (b if b.ndim == 2 else res_to_u64(b))
    bad = np.nonzero((a != b).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} of {len(a)} systems differ; first {bad[:4]}: {a[bad[:2]]} vs {b[bad[:2]]}"


def _run_device(dsm, eng, tr, cn):
    import torch
    n = tr.shape[0]
    st = torch.cuda.current_stream().cuda_stream
    dtr = torch.from_numpy(tr.view(np.int16)).cuda()
    dcn = torch.from_numpy(cn.view(np.int32)).cuda()
    out = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
    cnt = torch.zeros(pydsm.NCOUNTERS, dtype=torch.int64, device="cuda")
    eng.run_packed_device(dtr.data_ptr(), dcn.data_ptr(), n, out.data_ptr(), cnt.data_ptr(), st)
    torch.cuda.synchronize()
    return (out.cpu().numpy().view(dsm.RESULT_DTYPE).reshape(-1),
            dsm.counters_to_dict(cnt.cpu().numpy().view(np.uint64)))


def test_assert_failed_home_beyond_np(dsm, orc):
    """4-node device traces with some addresses homed at nodes 4-7: those systems end with
    ASSERT_FAILED in the round of the offending issue, the others run normally."""
    n = 2048
    tr, cn = orc.generate(4, "uniform", 31, 64, 0, n)
    rng = np.random.default_rng(7)
    bad = rng.choice(n, n // 4, replace=False)
    for s in bad:
        nd, i = int(rng.integers(0, 4)), int(rng.integers(0, 64))
        tr[s, nd, i] = (tr[s, nd, i] & 0x80FF) | ((0x40 + int(rng.integers(0, 64))) << 8)
    ores, _ = orc.run_packed(4, tr, cn, nthreads=16)[:2]
    nasr = int(((ores["status"] & 0xFF) == 3).sum())
    assert nasr > 0
    with dsm.Engine(4, 64) as eng:
        res, cnt = _run_device(dsm, eng, tr, cn)
    _cmp(res, ores)
    assert cnt["status_ASSERT_FAILED"] == nasr
    # the host entry point validates instead (DSM_E_RANGE), as the CLI's loader does
    with dsm.Engine(4, 64) as eng:
        with pytest.raises(dsm.DsmError) as e:
            eng.run_packed(tr, cn)
        assert e.value.code == dsm.E_RANGE


def test_assert_failed_matches_reference_records(dsm, orc):
    """Final records of asserted systems: the other nodes finish the round's actions and
    nothing is delivered (oracle/ref_lockstep.c semantics)."""
    n = 256
    tr, cn = orc.generate(4, "uniform", 5, 64, 0, n)
    tr[:, 2, 10] = (tr[:, 2, 10] & 0x80FF) | (0x55 << 8)
    ores, _, _, ofin = orc.run_packed(4, tr, cn, records=True, nthreads=16)
    with dsm.Engine(4, 64, snapshots=True) as eng:
        res, _ = _run_device(dsm, eng, tr, cn)
        for s in range(0, n, 17):
            for nd in range(4):
                assert np.array_equal(eng.node_state(s, nd)[1], ofin[s, nd])
    _cmp(res, ores)
    assert ((res["status"] & 0xFF) == 3).sum() > 0


def test_device_counts_are_clamped(dsm, orc):
    n = 128
    tr, cn = orc.generate(8, "uniform", 2, 64, 0, n)
    cn2 = cn.copy()
    cn2[::3, 1] = 1000                       # above max_instr (64): clamped to 64
    ores, _ = orc.run_packed(8, tr, np.minimum(cn2, 64), nthreads=16)[:2]
    with dsm.Engine(8, 64) as eng:
        res, _ = _run_device(dsm, eng, tr, cn2)
    _cmp(res, ores)


@pytest.mark.parametrize("limit_log2", [7, 9])
def test_round_limit_message_bound(dsm, orc, limit_log2):
    n = 4096
    orc.set_round_limit(1 << limit_log2)
    try:
        ores, _ = orc.run_generated(8, "uniform", 4, 4096, 0, n, nthreads=16)
        tr, cn = orc.generate(8, "uniform", 4, 4096, 0, 512)
        pres, _ = orc.run_packed(8, tr, cn, nthreads=16)[:2]
    finally:
        orc.set_round_limit(0)
    with dsm.Engine(8, 4096, type_counts=True) as eng:
        eng.set_round_limit(limit_log2)
        res, cnt = eng.run_generated("uniform", 4, 4096, 0, n)
        pk, _ = eng.run_packed(tr, cn)
    _cmp(res, ores)
    _cmp(pk, pres)
    assert cnt["status_ROUND_LIMIT"] == int(((ores["status"] & 0xFF) == 4).sum()) > 0


@pytest.mark.parametrize("cap,ring", [(3, 12), (6, 4), (5, 8)])
def test_ring_overflow_beyond_inbox_limit(dsm, orc, cap, ring):
    """Inbox limit below the fast ring (reported by the fast kernel's hand-off + 256-deep
    re-run) and above it (the re-run sees the deeper inbox first)."""
    n = 8192
    ores, _ = orc.run_generated(8, "uniform", 6, 4096, 0, n, ring_cap=cap, nthreads=16)
    novf = int(((ores["status"] & 0xFF) == 2).sum())
    assert novf > 0
    with dsm.Engine(8, 4096, ring_cap=ring) as eng:
        eng.set_inbox_limit(cap)
        res, cnt = eng.run_generated("uniform", 6, 4096, 0, n)
        tr, cn = orc.generate(8, "uniform", 6, 4096, 0, 1024)
        pk, _ = eng.run_packed(tr, cn)
    _cmp(res, ores)
    _cmp(pk, ores[:1024])
    assert cnt["status_RING_OVERFLOW"] == novf


def test_ring_overflow_matches_reference_text(dsm, orc):
    """The same inbox limit on the reference's own handler text (oracle/_ref, where built):
    its harness's staged delivery applies the cap (DSM_REF_INBOX_LIMIT)."""
    b = os.path.join(ORACLE, "_ref", "ref_lockstep_np8")
    if not os.path.exists(b):
        pytest.skip("oracle/_ref not built")
    n = 512
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "r.bin")
        subprocess.run([b, "gen", "0", "6", "4096", "0", str(n), out], check=True,
                       env=dict(os.environ, DSM_REF_INBOX_LIMIT="3"))
        raw = np.fromfile(out, dtype=np.uint8).reshape(n, 32 + 2 * 8 * 64)
    ref = raw[:, :32].copy().view(orc.RES_DT).reshape(-1)
    assert ((ref["status"] & 0xFF) == 2).sum() > 0
    with dsm.Engine(8, 4096) as eng:
        eng.set_inbox_limit(3)
        res, _ = eng.run_generated("uniform", 6, 4096, 0, n)
    _cmp(res, ref)
