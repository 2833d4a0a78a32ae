"""printProcessorState text (assignment.c:824-876) on the CPU side: the oracle's clean-room
formatter and the host boundary helper dsm_format_dump against the reference's OWN
printProcessorState output (md5 per record, tests/golden/dumps, made by
oracle/_ref/ref_lockstep_np8 fmt) for 4096 seeded random node records."""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLD


@pytest.fixture(scope="module")
def gold():
    recs = np.load(os.path.join(GOLD, "dumps", "random_recs.npy"))
    with open(os.path.join(GOLD, "dumps", "random_md5.json")) as f:
        meta = json.load(f)
    return recs, meta["texts"], meta["np"]


def _md5(s):
    return hashlib.md5(s.encode()).hexdigest()


def test_fixture_covers_every_cache_state_count(gold):
    recs, texts, _ = gold
    n_excl = (recs[:, 56:60] == 1).sum(axis=1)
    assert set(n_excl.tolist()) == {0, 1, 2, 3, 4}
    assert [t["len"] for t in texts] == (1954 + n_excl).tolist()


def test_oracle_formatter_matches_reference(gold):
    import pyoracle
    recs, texts, np_ = gold
    for k in range(len(recs)):
        s = pyoracle.format_dump(k % np_, recs[k])
        assert (len(s), _md5(s)) == (texts[k]["len"], texts[k]["md5"]), k


def test_host_formatter_matches_reference(gold):
    import pydsm
    recs, texts, np_ = gold
    for k in range(len(recs)):
        s = pydsm.format_dump(k % np_, recs[k])
        assert (len(s), _md5(s)) == (texts[k]["len"], texts[k]["md5"]), k
