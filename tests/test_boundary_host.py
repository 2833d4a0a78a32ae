"""Host side of the drop-in boundary (no GPU): libdsm.so loads and exports every symbol of
include/dsm.h; the trace parser follows initializeProcessor (assignment.c:802-818); the dump
formatter is byte-identical to printProcessorState (:824-876); the hash matches the oracle's.
"""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import pydsm
import pyoracle as orc
from conftest import PKG, REPO, TESTS, golden_dump, golden_records, inputs_dir


def header_functions():
    txt = open(os.path.join(REPO, "include", "dsm.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:[\w\s\*]+?)\b(dsm_\w+)\s*\(", txt, flags=re.M)))


def test_header_declares_expected_entry_points():
    fns = header_functions()
    for f in ["dsm_open", "dsm_close", "dsm_run_packed", "dsm_run_packed_device",
              "dsm_generate_device", "dsm_run_generated", "dsm_run_generated_device",
              "dsm_get_node_state", "dsm_parse_trace_file", "dsm_load_test_dir",
              "dsm_format_dump", "dsm_write_dump", "dsm_node_hash", "dsm_strerror"]:
        assert f in fns


def test_library_exports_every_header_symbol():
    L = pydsm.lib()
    missing = [f for f in header_functions() if not hasattr(L, f)]
    assert not missing, missing
    out = subprocess.run(["nm", "-D", "--defined-only", pydsm.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if " T " in l}
    assert set(header_functions()) <= exported


def _struct_fields(name):
    txt = open(os.path.join(REPO, "include", "dsm.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    body = re.search(r"typedef struct %s \{(.*?)\} %s;" % (name, name), txt, flags=re.S).group(1)
    return re.findall(r"\b(\w+)\s*;", body)


def test_launch_info_binding_matches_header():
    """pydsm's ctypes mirror of dsm_launch_info (ABI 4) has the header's fields in order,
    all of them int, so the library never writes past the caller's struct."""
    assert [f for f, _ in pydsm.LaunchInfo._fields_] == _struct_fields("dsm_launch_info")
    assert ctypes.sizeof(pydsm.LaunchInfo) == 4 * len(_struct_fields("dsm_launch_info"))
    assert set(pydsm.RESUME_FORMS) == {0, 1, 2, 3}


def test_counter_binding_matches_header():
    """dsm_counters (ABI 4: DSM_NCOUNTERS slots) and pydsm.COUNTER_FIELDS agree slot by slot;
    ff_passes (hit-run fast-forward steps) and ser_macro_steps (the serial pass's lone-node
    transaction steps) are separate slots."""
    txt = open(os.path.join(REPO, "include", "dsm.h")).read()
    n = int(re.search(r"#define DSM_NCOUNTERS (\d+)", txt).group(1))
    assert n == pydsm.NCOUNTERS == len(pydsm.COUNTER_FIELDS)
    body = re.sub(r"/\*.*?\*/", "", re.search(r"typedef struct dsm_counters \{(.*?)\} dsm_counters;",
                                               txt, flags=re.S).group(1), flags=re.S)
    slots = []
    for name, arr in re.findall(r"uint64_t (\w+)(?:\[(\w+)\])?;", body):
        k = 13 if arr == "DSM_NTYPES" else (int(arr) if arr else 1)
        slots += [name] * k
    assert len(slots) == n
    for i, f in enumerate(pydsm.COUNTER_FIELDS):
        want = {"msgs_by_type": "msgs_", "by_status": "status_", "reserved": "reserved_"}.get(slots[i], slots[i])
        assert f.startswith(want), (i, f, slots[i])
    assert pydsm.COUNTER_FIELDS[pydsm.MAX_SLOT] == "max_rounds"


def _li(**kw):
    li = pydsm.LaunchInfo()
    base = dict(np=8, ring_cap=12, block_threads=256, gen=0, occ=5, budget_mode=48, resume_mode=-1,
                ser_cap=0, resume_form=2)
    for k, v in dict(base, **kw).items():
        setattr(li, k, v)
    return li


@pytest.mark.parametrize("kw,want", [
    ({}, "budget=sim_kernel<8, 12, 4, false, 48, 5> resume=ser_kernel<8, false>"),
    (dict(ser_cap=1, np=4, budget_mode=8, resume_form=2),
     "budget=sim_kernel<4, 12, 4, false, 8, 5> resume=ser_kernel<4, true>"),
    (dict(budget_mode=16, resume_mode=0, resume_form=3),
     "budget=sim_kernel<8, 12, 4, false, 16, 5> resume=sim_kernel<8, 12, 4, false, 0, 5>"),
    (dict(budget_mode=0, gen=1, resume_form=0, ring_cap=4), "run=sim_kernel<8, 4, 4, true, 0, 5>"),
    (dict(budget_mode=-1, resume_form=0), "none"),
])
def test_launch_kernel_names(kw, want):
    """dsm_launch_kernel_names (host only): the measurement label of the kernels that ran."""
    L = pydsm.lib()
    buf = ctypes.create_string_buffer(256)
    n = L.dsm_launch_kernel_names(ctypes.byref(_li(**kw)), buf, 256)
    assert buf.raw[:n].decode() == want
    assert L.dsm_launch_kernel_names(ctypes.byref(_li(**kw)), buf, len(want)) == pydsm.E_INVAL   # no room for the NUL


def test_abi_version_and_errors():
    L = pydsm.lib()
    assert L.dsm_abi_version() == 5
    # the header, the library and the driver's build() check agree on the ABI version
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    hdr = open(os.path.join(root, "include", "dsm.h")).read()
    assert re.search(r"#define DSM_ABI_VERSION\s+5\b", hdr)
    assert "dsm_abi_version() == 5" in open(os.path.join(root, "__graft_entry__.py")).read()
    assert pydsm.strerror(0) == "ok"
    for code in range(-7, 0):
        assert pydsm.strerror(code) != "unknown error"


@pytest.mark.parametrize("test", TESTS)
def test_parser_reads_reference_inputs(test):
    for core in range(4):
        p = os.path.join(inputs_dir(test), f"core_{core}.txt")
        mine = pydsm.parse_trace_file(p, 32)
        ref = orc.parse_core_file(p, 32)
        assert list(mine) == ref


def _write(tmp_path, name, text):
    p = tmp_path / name
    p.write_bytes(text.encode())
    return str(p)


def test_parser_semantics(tmp_path):
    # %hhu wraps modulo 256 and %hhx takes the 0x prefix (:807, :812)
    p = _write(tmp_path, "a.txt", "WR 0x15 300\nRD 0x17\nWR 0x01 255\n")
    got = pydsm.parse_trace_file(p, 32)
    assert list(got) == [pydsm.pack_instr("W", 0x15, 300 % 256), pydsm.pack_instr("R", 0x17),
                         pydsm.pack_instr("W", 0x01, 255)]
    # more than MAX_INSTR_NUM lines are silently truncated (:805)
    p = _write(tmp_path, "b.txt", "".join(f"RD 0x{i % 64:02X}\n" for i in range(40)))
    assert len(pydsm.parse_trace_file(p, 32)) == 32
    assert len(pydsm.parse_trace_file(p, 64)) == 40
    # empty file: zero instructions (tests/sample/core_2.txt)
    assert len(pydsm.parse_trace_file(_write(tmp_path, "c.txt", ""), 32)) == 0
    # a chunk that is neither RD nor WR: the reference would count garbage -> rejected
    with pytest.raises(pydsm.DsmError) as e:
        pydsm.parse_trace_file(_write(tmp_path, "d.txt", "RD 0x01\n\nRD 0x02\n"), 32)
    assert e.value.code == pydsm.E_FORMAT
    # missing file (:796-800)
    with pytest.raises(pydsm.DsmError) as e:
        pydsm.parse_trace_file(str(tmp_path / "nope.txt"), 32)
    assert e.value.code == pydsm.E_IO
    # addresses beyond 8 nodes cannot be simulated (bitVector is one byte)
    with pytest.raises(pydsm.DsmError) as e:
        pydsm.parse_trace_file(_write(tmp_path, "e.txt", "RD 0x90\n"), 32)
    assert e.value.code == pydsm.E_RANGE


def test_load_test_dir_range_check(tmp_path):
    d = tmp_path / "tests" / "t"
    d.mkdir(parents=True)
    for n in range(8):
        (d / f"core_{n}.txt").write_text("RD 0x45\n" if n == 0 else "")
    tr = np.zeros((8, 32), dtype=np.uint16)
    cn = np.zeros(8, dtype=np.uint32)
    cwd = os.getcwd()
    try:
        os.chdir(tmp_path)
        rc = pydsm.lib().dsm_load_test_dir(b"t", 4, 32, ctypes.c_void_p(tr.ctypes.data), 32,
                                          ctypes.c_void_p(cn.ctypes.data))
        assert rc == pydsm.E_RANGE      # home node 4 does not exist with NUM_PROCS=4
        rc = pydsm.lib().dsm_load_test_dir(b"t", 8, 32, ctypes.c_void_p(tr.ctypes.data), 32,
                                          ctypes.c_void_p(cn.ctypes.data))
        assert rc == 0 and cn[0] == 1
    finally:
        os.chdir(cwd)


@pytest.mark.parametrize("test", TESTS)
def test_formatter_byte_exact(test):
    recs = golden_records(test)
    for core in range(4):
        assert pydsm.format_dump(core, recs[0, core]) == golden_dump(test, core)


def test_write_dump(tmp_path):
    recs = golden_records("test_4")
    rc = pydsm.lib().dsm_write_dump(3, ctypes.c_void_p(recs[0, 3].ctypes.data), str(tmp_path).encode())
    assert rc == 0
    assert (tmp_path / "core_3_output.txt").read_text() == golden_dump("test_4", 3)


def test_hash_matches_oracle():
    rng = np.random.default_rng(0)
    for _ in range(50):
        rec = rng.integers(0, 256, 64, dtype=np.uint8)
        node = int(rng.integers(0, 8))
        for nw in (15, 16):
            assert pydsm.node_hash(node, rec, nw) == orc.hash_rec(node, rec, nw)


def test_no_gpu_means_loud_failure():
    """Without a usable gfx950 the engine refuses to run (no CPU fallback)."""
    if pydsm.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(pydsm.DsmError) as e:
        pydsm.Engine(8, 64)
    assert e.value.code == pydsm.E_DEVICE


def test_cli_without_gpu_fails_loudly(tmp_path):
    if pydsm.device_count() > 0:
        pytest.skip("a GPU is visible")
    os.symlink(os.path.join(REPO, "tests", "golden", "inputs"), tmp_path / "tests")
    r = subprocess.run([pydsm.CLI_PATH, "sample"], cwd=tmp_path, capture_output=True, text=True)
    assert r.returncode == 1
    assert "dsm_open" in r.stderr
    assert r.stdout == ""        # the core files are scanned on the GPU: nothing initialised
    assert not list(tmp_path.glob("core_*_output.txt"))


def test_cli_usage_and_missing_input(tmp_path):
    r = subprocess.run([pydsm.CLI_PATH], capture_output=True, text=True)
    assert r.returncode == 1 and "Usage" in r.stderr
    r = subprocess.run([pydsm.CLI_PATH, "nosuch"], cwd=tmp_path, capture_output=True, text=True)
    assert r.returncode == 1
    assert "Error: could not open file tests/nosuch/core_0.txt" in r.stderr
