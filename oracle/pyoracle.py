"""oracle/pyoracle.py -- TEST INFRASTRUCTURE ONLY.

ctypes wrapper of oracle/liboracle.so (the clean-room C restatement, dsm_oracle.c).  Only
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module, and
only as the checker / the timed CPU baseline -- never as the thing measured or shipped.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")
RES_DT = np.dtype([("status", "<u4"), ("rounds", "<u4"), ("msgs", "<u4"), ("instrs", "<u4"),
                   ("dump_hash", "<u8"), ("final_hash", "<u8")])
DIST = {"uniform": 0, "hot": 1, "evict": 2}
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.run(["make", "-C", HERE, "liboracle.so"], check=True,
                           stdout=subprocess.DEVNULL)
        L = ctypes.CDLL(LIB)
        vp, u64, u32, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
        L.orc_run_system.argtypes = [i32, vp, vp, u32, u32, vp, vp, vp, vp]
        L.orc_run_packed.argtypes = [i32, vp, vp, u32, u64, u32, vp, vp, vp, vp, i32]
        L.orc_run_generated.argtypes = [i32, i32, u64, u32, u64, u64, u32, vp, vp, i32]
        L.orc_run_packed_ex.argtypes = [i32, vp, vp, u32, u64, u32, u64, u32, u64, vp, vp, vp, vp,
                                        u32, vp, i32]
        L.orc_generate.argtypes = [i32, i32, u64, u32, u64, u64, vp, vp]
        L.orc_generate.restype = None
        L.orc_format_dump.argtypes = [i32, vp, ctypes.c_char_p, i32]
        L.orc_hash_rec.argtypes = [i32, vp, i32]
        L.orc_hash_rec.restype = u64
        L.orc_set_round_limit.argtypes = [u32]
        L.orc_set_round_limit.restype = None
        _lib = L
    return _lib


def _p(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


def run_packed(np_, traces, counts, ring_cap=256, nthreads=8, records=False):
    """traces [n, np, stride] u16, counts [n, np] -> (results, by_type[13], dump, final)."""
    traces = np.ascontiguousarray(traces, dtype=np.uint16)
    counts = np.ascontiguousarray(counts, dtype=np.uint32)
    n, _, stride = traces.shape
    res = np.zeros(n, dtype=RES_DT)
    bt = np.zeros(13, dtype=np.uint64)
    dump = np.zeros((n, np_, 64), dtype=np.uint8) if records else None
    fin = np.zeros((n, np_, 64), dtype=np.uint8) if records else None
    rc = lib().orc_run_packed(np_, _p(traces), _p(counts), stride, n, ring_cap, _p(res), _p(dump),
                              _p(fin), _p(bt), nthreads)
    assert rc == 0
    return res, bt, dump, fin


LOCKSTEP = 0x10000


def run_packed_ex(np_, traces, counts, sched_seed=0, sched_thresh=LOCKSTEP, first_sys=0,
                  ring_cap=256, nthreads=8, issue=False):
    """run_packed with seeded schedule exploration (system id first_sys + i in the schedule
    hash) and, with issue=True, the issue order: (res, dump, fin, events [n, cap], n_events)."""
    traces = np.ascontiguousarray(traces, dtype=np.uint16)
    counts = np.ascontiguousarray(counts, dtype=np.uint32)
    n, _, stride = traces.shape
    res = np.zeros(n, dtype=RES_DT)
    dump = np.zeros((n, np_, 64), dtype=np.uint8)
    fin = np.zeros((n, np_, 64), dtype=np.uint8)
    cap = np_ * stride
    ev = np.zeros((n, cap), dtype=np.uint32) if issue else None
    evn = np.zeros(n, dtype=np.uint32) if issue else None
    rc = lib().orc_run_packed_ex(np_, _p(traces), _p(counts), stride, n, ring_cap, sched_seed,
                                 sched_thresh, first_sys, _p(res), _p(dump), _p(fin), _p(ev), cap,
                                 _p(evn), nthreads)
    assert rc == 0
    return res, dump, fin, ev, evn


def issue_lines(events):
    """DEBUG_INSTR lines (assignment.c:596-597) of one system's issue order."""
    out = []
    for e in events:
        node, ins = int(e) >> 16, int(e) & 0xFFFF
        out.append("Processor %d: instr type=%c, address=0x%02X, value=%d\n"
                   % (node, "W" if ins >> 15 else "R", (ins >> 8) & 0x7F, ins & 0xFF))
    return "".join(out)


def run_generated(np_, dist, seed, n_instr, first, n, ring_cap=256, nthreads=8):
    res = np.zeros(n, dtype=RES_DT)
    bt = np.zeros(13, dtype=np.uint64)
    rc = lib().orc_run_generated(np_, DIST.get(dist, dist), seed, n_instr, first, n, ring_cap,
                                 _p(res), _p(bt), nthreads)
    assert rc == 0
    return res, bt


def set_round_limit(limit):
    """Active rounds before ST_ROUND_LIMIT for the following runs (0 = default 2^22)."""
    lib().orc_set_round_limit(limit)


def generate(np_, dist, seed, n_instr, first, n):
    tr = np.zeros((n, np_, n_instr), dtype=np.uint16)
    cn = np.zeros((n, np_), dtype=np.uint32)
    lib().orc_generate(np_, DIST.get(dist, dist), seed, n_instr, first, n, _p(tr), _p(cn))
    return tr, cn


def format_dump(node, rec):
    rec = np.ascontiguousarray(rec, dtype=np.uint8)
    buf = ctypes.create_string_buffer(4096)
    n = lib().orc_format_dump(node, _p(rec), buf, 4096)
    assert n > 0
    return buf.raw[:n].decode()


def hash_rec(node, rec, nwords):
    rec = np.ascontiguousarray(rec, dtype=np.uint8)
    return int(lib().orc_hash_rec(node, _p(rec), nwords))


def parse_core_file(path, cap=32):
    """Plain-Python reading of a trace file with initializeProcessor's rules (:802-818),
    used to build oracle inputs for the shipped tests (RD/WR lines only)."""
    out = []
    with open(path, "rb") as f:
        data = f.read().decode()
    for line in data.splitlines(keepends=True):
        if len(out) >= cap:
            break
        parts = line.split()
        if parts[0] == "RD":
            out.append((0 << 15) | ((int(parts[1], 16) & 0xFF) << 8))
        elif parts[0] == "WR":
            out.append((1 << 15) | ((int(parts[1], 16) & 0xFF) << 8) | (int(parts[2]) & 0xFF))
        else:
            raise ValueError(line)
    return out


def load_test(inputs_dir, np_=4, stride=32, cap=32):
    tr = np.zeros((1, np_, stride), dtype=np.uint16)
    cn = np.zeros((1, np_), dtype=np.uint32)
    for n in range(np_):
        ins = parse_core_file(os.path.join(inputs_dir, f"core_{n}.txt"), cap)
        tr[0, n, :len(ins)] = ins
        cn[0, n] = len(ins)
    return tr, cn
