"""Per-quirk transition scenarios (tests/scenarios.py) on the oracle (CPU) and on the GPU
engine through the C ABI; the GPU results must also equal the oracle's bit for bit."""
import os
import subprocess
import tempfile

import numpy as np
import pytest

import pyoracle as orc
from conftest import ORACLE, res_to_u64
from scenarios import SCENARIOS


@pytest.mark.parametrize("name", sorted(SCENARIOS))
def test_scenario_oracle(name):
    tr, cn, check = SCENARIOS[name]()
    np_ = tr.shape[1]
    res, _, dump, fin = orc.run_packed(np_, tr, cn, records=True, nthreads=1)
    check(res[0], dump[0], fin[0])


def _ref_bin(np_):
    p = os.path.join(ORACLE, "_ref", f"ref_lockstep_np{np_}_i32" if np_ == 4 else f"ref_lockstep_np{np_}")
    return p if os.path.exists(p) else None


@pytest.mark.parametrize("name", sorted(SCENARIOS))
def test_scenario_reference_text(name):
    """Where oracle/_ref was built (build container), the reference's own handler text must
    agree with the hand-derived expectations too."""
    tr, cn, check = SCENARIOS[name]()
    np_ = tr.shape[1]
    b = _ref_bin(np_)
    if b is None:
        pytest.skip("oracle/_ref not built")
    with tempfile.TemporaryDirectory() as d:
        os.makedirs(os.path.join(d, "tests", "s"))
        for n in range(np_):
            with open(os.path.join(d, "tests", "s", f"core_{n}.txt"), "w") as f:
                for i in range(int(cn[0, n])):
                    w = int(tr[0, n, i])
                    f.write(f"WR 0x{(w >> 8) & 0x7F:02X} {w & 0xFF}\n" if w >> 15 else
                            f"RD 0x{(w >> 8) & 0x7F:02X}\n")
        subprocess.run([b, "tests", "s", "r.bin"], cwd=d, check=True, stdout=subprocess.DEVNULL)
        raw = np.fromfile(os.path.join(d, "r.bin"), dtype=np.uint8)
    res = raw[:32].view(orc.RES_DT)[0]
    recs = raw[32:].reshape(2, np_, 64)
    check(res, recs[0], recs[1])


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(SCENARIOS))
def test_scenario_gpu(name):
    import pydsm
    tr, cn, check = SCENARIOS[name]()
    np_ = tr.shape[1]
    with pydsm.Engine(np_, tr.shape[2], snapshots=True, type_counts=True) as eng:
        res, cnt = eng.run_packed(tr, cn)
        dump = np.stack([eng.node_state(0, n)[0] for n in range(np_)])
        fin = np.stack([eng.node_state(0, n)[1] for n in range(np_)])
    check(res[0], dump, fin)
    ores, obt, odump, ofin = orc.run_packed(np_, tr, cn, records=True, nthreads=1)
    assert np.array_equal(res_to_u64(res), res_to_u64(ores))
    mask = int(res[0]["status"]) >> 8
    for n in range(np_):
        if (mask >> n) & 1:
            assert np.array_equal(dump[n], odump[0, n])
        assert np.array_equal(fin[n], ofin[0, n])
    assert [cnt[k] for k in list(cnt)[:13]] == [int(x) for x in obt]
