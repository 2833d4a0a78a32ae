"""parse_kernel's branch-free chunk decoder (csrc/dsm_text.hip parse_fast_v3, and the earlier
word-parallel parse_fast_swar) against the byte-wise one they replaced in the chunk loop
(parse_fast): all cut from the kernel source and
compiled for the host, compared on 4M mutated canonical lines (reference: assignment.c:802-818,
fgets + sscanf("RD %hhx") / sscanf("WR %hhx %hhu"); the exact slow path takes what they decline)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "hp-assignment-2_amd", "csrc", "dsm_text.hip")


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_parse_fast_swar_matches_parse_fast(tmp_path):
    lines = open(SRC).read().split("\n")
    s = next(i for i, l in enumerate(lines) if l.startswith("DEVI uint32_t is_dec"))
    e = next(i for i, l in enumerate(lines) if l.startswith("#ifndef PARSE_SWAR"))
    (tmp_path / "pf.h").write_text("\n".join(lines[s:e]) + "\n")
    exe = tmp_path / "pfe"
    subprocess.run(["g++", "-O2", "-I", str(tmp_path), "-o", str(exe),
                    os.path.join(ROOT, "tests", "native", "parse_fast_equiv.cpp")], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and out.stdout.startswith("ok "), out.stdout + out.stderr
