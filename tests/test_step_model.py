"""Every row of the kernel's transition table (hp-assignment-2_amd/csrc/dsm_table.h) against
the oracle's handler, one action at a time (tests/model/step_model.cpp), on random node states
and messages -- including the rows no trace can reach, which therefore have no GPU scenario:
REPLY_ID at a line that no longer holds the block (assignment.c:339-346), EVICT_SHARED at a
non-home from a node that is not the home (:533-537) and the REPLY_WR / FLUSH_INVACK asserts
(:443, :489).  tools/find_scenarios.c (oracle branch probes over random systems) and the
probe counts over generated ensembles never reach them: a node holds one outstanding request
and only its replies install lines, so a reply always finds its block, and EVICT_SHARED is
only ever sent to the home or by the home."""
import json
import os
import subprocess

import pytest

from conftest import REPO


@pytest.fixture(scope="module")
def step_model(tmp_path_factory):
    d = tmp_path_factory.mktemp("sm")
    obj = str(d / "orc.o")
    subprocess.run(["gcc", "-O2", "-c", os.path.join(REPO, "oracle", "dsm_oracle.c"),
                    "-I", os.path.join(REPO, "oracle"), "-o", obj], check=True)
    exe = str(d / "step_model")
    subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", "-Wextra", "-Werror",
                    "-I", os.path.join(REPO, "oracle"),
                    "-I", os.path.join(REPO, "hp-assignment-2_amd", "csrc"),
                    os.path.join(REPO, "tests", "model", "step_model.cpp"), obj, "-o", exe],
                   check=True)
    return exe


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_every_table_row_matches_the_handler(step_model, seed):
    r = subprocess.run([step_model, "200000", str(seed)], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr
    d = json.loads(r.stdout)
    assert d["rows_hit"] >= 170
    assert all(k > 10000 for k in d["kinds"])          # every type and both issue ops
    for row in ("rid_mismatch", "evs_not_from_home", "rwr_assert", "flinv_assert"):
        assert d[row] > 1000, row
