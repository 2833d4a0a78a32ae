"""The chunk parser of the gfx950 trace parser (hp-assignment-2_amd/csrc/dsm_parse.h: one
fgets chunk of initializeProcessor, assignment.c:802-818) checked on the CPU against glibc's
own sscanf("RD %hhx") / sscanf("WR %hhx %hhu") over fuzzed chunks: well-formed lines like the
shipped tests, token soups (signs, 0x prefixes, whitespace kinds, wrap-around and overflowing
numbers, truncation at 19 bytes) and random bytes."""
import os
import subprocess

import pytest

from conftest import REPO

SRC = os.path.join(REPO, "tests", "model", "parse_model.cpp")


@pytest.fixture(scope="module")
def model(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("pm") / "parse_model")
    subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", "-Wextra", "-Werror",
                    "-I", os.path.join(REPO, "hp-assignment-2_amd", "csrc"), SRC, "-o", exe],
                   check=True)
    return exe


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_chunk_parser_equals_glibc_sscanf(model, seed):
    out = subprocess.run([model, "fuzz", str(seed), "400000"], check=True, capture_output=True,
                         text=True)
    bad, ok, fmt, rng = map(int, out.stdout.split())
    assert bad == 0, out.stderr
    assert ok > 50000 and fmt > 50000 and rng > 10000   # every outcome well exercised
