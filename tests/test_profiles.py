"""CPU: the profile-derived fields of the bench line (profiles/pmc_issue.json, the compute-side
roof of the transition kernels; profiles/pmc_traffic.json, their HBM traffic) are what the
committed rocprofv3 passes say: recomputed here from the raw counter CSVs they cite."""
import json
import os
import sys

import pytest

from conftest import REPO

sys.path.insert(0, os.path.join(REPO, "tools"))

ISSUE = json.load(open(os.path.join(REPO, "profiles", "pmc_issue.json")))
CASES = [(c, k) for c, v in sorted(ISSUE.items()) for k in sorted(v)]


@pytest.mark.parametrize("config,kernel", CASES)
def test_issue_metrics_match_the_counters(config, kernel):
    import issue
    e = ISSUE[config][kernel]
    d = e["source"].split("/pmc_sq")[0]
    if not os.path.isdir(os.path.join(REPO, d)):
        pytest.skip(f"{d} not present")
    again = issue.summarize(os.path.join(REPO, d), issue.KERNELS[kernel])
    for k in ("valu_busy", "waves_per_simd", "wait_frac", "issue_stall_frac", "clock_ghz", "ms"):
        assert again[k] == e[k], k
    # by hand, from the first dispatch's raw counters: VALU x 2 / (GRBM / 8 x 1024)
    sq = issue.dispatches(os.path.join(REPO, d, "pmc_sq"), issue.KERNELS[kernel])
    wall, c = next(iter(sq.values()))
    busy = c["SQ_INSTS_VALU"] * 2 / (c["GRBM_GUI_ACTIVE"] / 8 * 1024)
    assert 0.0 < busy < 1.0 and abs(busy - e["valu_busy"]) < 0.05
    assert 0.5 < e["waves_per_simd"] <= 8 and 0 < e["wait_frac"] < 1


def test_every_bench_config_has_issue_metrics():
    for c in ("random", "hot", "evict"):
        assert "sim_kernel_budget" in ISSUE[c]
        assert ("ser_kernel" in ISSUE[c]) or ("sim_kernel_ff" in ISSUE[c])
