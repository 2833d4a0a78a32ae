import json
import os
import subprocess
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "hp-assignment-2_amd")
ORACLE = os.path.join(REPO, "oracle")
GOLD = os.path.join(REPO, "tests", "golden")
TESTS = ["sample", "test_1", "test_2", "test_3", "test_4"]

for p in (PKG, ORACLE):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


def _build():
    """Build the in-tree libraries if they are missing (hipcc cross-compiles without a GPU)."""
    if not os.path.exists(os.path.join(ORACLE, "liboracle.so")):
        subprocess.run(["make", "-C", ORACLE, "liboracle.so"], check=True, stdout=subprocess.DEVNULL)
    if not all(os.path.exists(os.path.join(PKG, f)) for f in ("libdsm.so", "cache_simulator",
                                                                "dsm_ensemble")):
        subprocess.run(["make", "-C", PKG, "-j4"], check=True, stdout=subprocess.DEVNULL)


_build()


@pytest.fixture(scope="session")
def summary():
    with open(os.path.join(GOLD, "lockstep", "summary.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def ensemble_meta():
    with open(os.path.join(GOLD, "ensemble", "meta.json")) as f:
        return json.load(f)


def golden_aggregate(name):
    """Full-size aggregates of the reference's handler text (oracle/gen_fixtures.py aggregates)."""
    with open(os.path.join(GOLD, "aggregates.json")) as f:
        return json.load(f)[name]


def golden_dump(test, core):
    p = os.path.join(GOLD, "lockstep", test, f"core_{core}_output.txt")
    return open(p).read() if os.path.exists(p) else None


def golden_records(test):
    return np.load(os.path.join(GOLD, "lockstep", test, "records.npy"))  # [2, np, 64]


def golden_ensemble(name):
    return np.load(os.path.join(GOLD, "ensemble", f"{name}.npy"))  # [n, 6] u64


def golden_ensemble_recs(name):
    return np.load(os.path.join(GOLD, "ensemble", f"{name}_recs.npy"))  # [16, 2, np, 64]


def res_to_u64(r):
    return np.stack([r["status"].astype(np.uint64), r["rounds"].astype(np.uint64),
                     r["msgs"].astype(np.uint64), r["instrs"].astype(np.uint64),
                     r["dump_hash"], r["final_hash"]], axis=1)


def inputs_dir(test):
    return os.path.join(GOLD, "inputs", test)
