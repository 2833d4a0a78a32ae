"""pydsm -- thin ctypes binding of libdsm.so (include/dsm.h) for tests, bench.py and smoke().

This is plumbing, not the product: the engine is the C ABI over the gfx950 HIP kernels.
There is deliberately no fallback of any kind: if libdsm.so is missing, or the device is not
a gfx950, every engine call raises DsmError.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DSM_LIB") or os.path.join(HERE, "libdsm.so")   # DSM_LIB: A/B builds
CLI_PATH = os.path.join(HERE, "cache_simulator")

NTYPES = 13
TYPE_NAMES = ["READ_REQUEST", "WRITE_REQUEST", "REPLY_RD", "REPLY_WR", "REPLY_ID", "INV",
              "UPGRADE", "WRITEBACK_INV", "WRITEBACK_INT", "FLUSH", "FLUSH_INVACK",
              "EVICT_SHARED", "EVICT_MODIFIED"]
STATUS_NAMES = ["COMPLETED", "DEADLOCKED", "RING_OVERFLOW", "ASSERT_FAILED", "ROUND_LIMIT"]
DIST = {"uniform": 0, "hot": 1, "evict": 2}
FF_OFF, FF_ON, FF_AUTO = 0, 1, 2             # dsm_set_fast_forward
F_SNAPSHOTS = 1
F_TIMING = 2
F_TYPE_COUNTS = 4
F_ISSUE_TRACE = 8
SCHED_LOCKSTEP = 0x10000

RESULT_DTYPE = np.dtype([("status", "<u4"), ("rounds", "<u4"), ("msgs", "<u4"),
                         ("instrs", "<u4"), ("dump_hash", "<u8"), ("final_hash", "<u8")])
COUNTER_FIELDS = ([f"msgs_{t}" for t in TYPE_NAMES] +
                  ["msgs", "instrs", "rounds", "systems"] +
                  [f"status_{s}" for s in STATUS_NAMES] +
                  ["sum_dump_hash", "sum_final_hash", "max_rounds", "overflow_reruns",
                   "wave_rounds", "resumed", "ff_passes", "ff_steps", "ff_sample_instrs",
                   "ff_sample_runs", "ser_macro_steps", "ser_iterations"] +
                  [f"reserved_{i}" for i in range(6)])
NCOUNTERS = 40                               # DSM_NCOUNTERS (ABI 4; ser_iterations: ABI 5)
assert len(COUNTER_FIELDS) == NCOUNTERS
MAX_SLOT = COUNTER_FIELDS.index("max_rounds")   # the one counter that is a max, not a sum

DUMP_BASE, DUMP_MAX, DUMP_SLOT = 1954, 1958, 1968
VIEW_DUMP, VIEW_FINAL = 0, 1
E_INVAL, E_DEVICE, E_NOMEM, E_IO, E_FORMAT, E_STATE, E_RANGE = -1, -2, -3, -4, -5, -6, -7


class DsmError(RuntimeError):
    def __init__(self, code, what):
        self.code = code
        super().__init__(f"{what}: {strerror(code)} ({code})")


class Config(ctypes.Structure):
    _fields_ = [("np", ctypes.c_int), ("max_instr", ctypes.c_uint32),
                ("ring_cap", ctypes.c_uint32), ("flags", ctypes.c_uint32)]


class Gen(ctypes.Structure):
    _fields_ = [("seed", ctypes.c_uint64), ("dist", ctypes.c_int), ("n_instr", ctypes.c_uint32)]


class LaunchInfo(ctypes.Structure):
    _fields_ = [("grid_blocks", ctypes.c_int), ("block_threads", ctypes.c_int),
                ("waves_per_cu", ctypes.c_int), ("cus", ctypes.c_int),
                ("ring_cap", ctypes.c_int), ("lds_bytes_per_block", ctypes.c_int),
                ("resume_blocks", ctypes.c_int), ("budget_log2", ctypes.c_int),
                ("late_log2", ctypes.c_int), ("round_limit_log2", ctypes.c_int),
                ("fmt_tile", ctypes.c_int), ("parse_bpl", ctypes.c_int),
                ("resume_form", ctypes.c_int), ("budget_rounds", ctypes.c_int),
                ("ff_picked", ctypes.c_int), ("np", ctypes.c_int), ("gen", ctypes.c_int),
                ("occ", ctypes.c_int), ("budget_mode", ctypes.c_int),
                ("resume_mode", ctypes.c_int), ("ser_cap", ctypes.c_int)]


RESUME_FORMS = {0: "none", 1: "lock-step", 2: "serial", 3: "fast-forward lock-step"}


_lib = None


def lib():
    """Load libdsm.so (raises if it has not been built: there is no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise OSError(f"{LIB_PATH} not built (run `make -C hp-assignment-2_amd`)")
        # torch (ROCm build) bundles its own libamdhip64.so.7 / libhsa-runtime64.so.1.  A
        # process must hold ONE HIP runtime: load torch's first so libdsm's DT_NEEDED entries
        # (same sonames) bind to it and device pointers / streams are shared with torch.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        vp, u64, u32, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
        sig = {
            "dsm_abi_version": (i32, []),
            "dsm_strerror": (ctypes.c_char_p, [i32]),
            "dsm_device_count": (i32, [ctypes.POINTER(i32)]),
            "dsm_open": (i32, [i32, ctypes.POINTER(Config), ctypes.POINTER(vp)]),
            "dsm_close": (None, [vp]),
            "dsm_launch_info_get": (i32, [vp, ctypes.POINTER(LaunchInfo)]),
            "dsm_launch_kernel_names": (i32, [ctypes.POINTER(LaunchInfo), ctypes.c_char_p,
                                              ctypes.c_size_t]),
            "dsm_run_packed": (i32, [vp, vp, vp, u64, vp, vp]),
            "dsm_run_packed_device": (i32, [vp, vp, vp, u64, vp, vp, vp]),
            "dsm_generate_device": (i32, [vp, ctypes.POINTER(Gen), u64, u64, vp, vp, vp]),
            "dsm_run_generated_device": (i32, [vp, ctypes.POINTER(Gen), u64, u64, vp, vp, vp]),
            "dsm_run_generated": (i32, [vp, ctypes.POINTER(Gen), u64, u64, vp, vp]),
            "dsm_get_node_state": (i32, [vp, u64, i32, vp, vp]),
            "dsm_last_kernel_ms": (i32, [vp, ctypes.POINTER(ctypes.c_float)]),
            "dsm_kernel_ms_history": (i32, [vp, vp, u32, ctypes.POINTER(u32)]),
            "dsm_set_budget": (i32, [vp, u32, u32]),
            "dsm_set_round_limit": (i32, [vp, u32]),
            "dsm_set_inbox_limit": (i32, [vp, u32]),
            "dsm_set_fast_forward": (i32, [vp, i32]),
            "dsm_parse_trace_file": (i32, [ctypes.c_char_p, vp, u32, ctypes.POINTER(u32)]),
            "dsm_load_test_dir": (i32, [ctypes.c_char_p, i32, u32, vp, u32, vp]),
            "dsm_format_dump": (i32, [i32, vp, ctypes.c_char_p, ctypes.c_size_t]),
            "dsm_write_dump": (i32, [i32, vp, ctypes.c_char_p]),
            "dsm_node_hash": (u64, [i32, vp, i32]),
            "dsm_format_dumps_device": (i32, [vp, vp, u32, u64, vp, vp, vp]),
            "dsm_format_run_dumps_device": (i32, [vp, i32, u64, u64, vp, vp, vp]),
            "dsm_write_run_dumps": (i32, [vp, u64, u32, ctypes.c_char_p]),
            "dsm_set_schedule": (i32, [vp, u64, u32]),
            "dsm_get_issue_trace": (i32, [vp, u64, vp, u32, ctypes.POINTER(u32)]),
            "dsm_format_issue_trace": (i32, [vp, u32, ctypes.c_char_p, ctypes.c_size_t]),
            "dsm_parse_traces_device": (i32, [vp, vp, vp, u64, u32, vp, vp, vp, vp]),
            "dsm_parse_traces": (i32, [vp, vp, vp, u64, u32, vp, vp, vp]),
            "dsm_generate_text_device": (i32, [vp, ctypes.POINTER(Gen), u64, u64, vp, vp, vp]),
            # ABI 5: per-system aggregates and the multi-GPU group (RCCL)
            "dsm_aggregate_device": (i32, [vp, vp, u64, u64, vp, vp]),
            "dsm_aggregate_results": (i32, [vp, u64, u64, vp]),
            "dsm_result_digest": (u64, [u64, vp]),
            "dsm_group_unique_id": (i32, [vp]),
            "dsm_group_init_rank": (i32, [i32, i32, i32, vp, ctypes.POINTER(vp)]),
            "dsm_group_init_all": (i32, [i32, vp, vp]),
            "dsm_group_info": (i32, [vp, ctypes.POINTER(i32), ctypes.POINTER(i32), ctypes.POINTER(i32)]),
            "dsm_group_close": (i32, [vp]),
            "dsm_group_allreduce": (i32, [vp, vp, ctypes.c_size_t, i32, vp]),
            "dsm_group_allreduce_counters": (i32, [vp, vp, vp]),
            "dsm_group_allreduce_aggregate": (i32, [vp, vp, vp]),
            "dsm_group_barrier": (i32, [vp, vp]),
        }
        for name, (res, args) in sig.items():
            if os.environ.get("DSM_LIB") and not hasattr(L, name):
                continue        # an older A/B build without this entry point
            f = getattr(L, name)
            f.restype, f.argtypes = res, args
        _lib = L
    return _lib


def strerror(code):
    try:
        return lib().dsm_strerror(code).decode()
    except OSError:
        return "libdsm.so unavailable"


def _check(rc, what):
    if rc != 0:
        raise DsmError(rc, what)


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


COUNTERS_BYTES = NCOUNTERS * 8
NAGG = 16                                    # DSM_NAGG (ABI 5)
AGG_FIELDS = ("systems", "msgs", "instrs", "rounds", "max_rounds", "st0", "st1", "st2", "st3",
              "st4", "sum_dump_hash", "sum_final_hash", "result_digest", "reserved0",
              "reserved1", "reserved2")
assert len(AGG_FIELDS) == NAGG
RED_SUM, RED_MAX = 0, 1


def _dptr(x, min_bytes=0):
    """A device pointer argument: an int (raw pointer, unchecked), None, or a tensor, whose
    size is checked against min_bytes (a dsm_counters buffer of an older ABI is too small)."""
    if x is None:
        return None
    if hasattr(x, "data_ptr"):
        nb = x.numel() * x.element_size()
        if nb < min_bytes:
            raise DsmError(-1, f"device buffer of {nb} bytes, needs {min_bytes}")
        return ctypes.c_void_p(x.data_ptr())
    return ctypes.c_void_p(x)


def agg_vec_to_dict(v):
    """A dsm_aggregate (DSM_NAGG uint64) as the golden-aggregate dict (tests/golden/aggregates.json)."""
    v = [int(x) for x in np.asarray(v, dtype=np.uint64).reshape(-1)]
    a = dict(zip(AGG_FIELDS, v))
    out = {k: a[k] for k in ("systems", "msgs", "instrs", "rounds", "max_rounds")}
    out["status"] = [a[f"st{i}"] for i in range(5)]
    out.update({k: "0x%016x" % a[k] for k in ("sum_dump_hash", "sum_final_hash", "result_digest")})
    return out


def aggregate_results_c(res, first_idx=0):
    """dsm_aggregate_results (the library's host fold) of per-system results, as a dict."""
    res = np.ascontiguousarray(res).view(RESULT_DTYPE).reshape(-1)
    out = np.zeros(NAGG, dtype=np.uint64)
    _check(lib().dsm_aggregate_results(_ptr(res), len(res), first_idx, _ptr(out)),
           "dsm_aggregate_results")
    return agg_vec_to_dict(out)


class Group:
    """dsm_group: one RCCL communicator per GPU for the end-of-run all-reduces (ABI 5).
    Rank 0 makes the id (Group.unique_id()) and hands it to every rank out of band."""

    @staticmethod
    def unique_id():
        b = (ctypes.c_ubyte * 128)()
        _check(lib().dsm_group_unique_id(b), "dsm_group_unique_id")
        return bytes(b)

    def __init__(self, device, nranks, rank, uid):
        assert len(uid) == 128
        self.g = ctypes.c_void_p()
        b = (ctypes.c_ubyte * 128).from_buffer_copy(uid)
        _check(lib().dsm_group_init_rank(device, nranks, rank, b, ctypes.byref(self.g)),
               "dsm_group_init_rank")

    def info(self):
        r, n, d = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        _check(lib().dsm_group_info(self.g, ctypes.byref(r), ctypes.byref(n), ctypes.byref(d)),
               "dsm_group_info")
        return r.value, n.value, d.value

    def allreduce(self, d_buf, n, op=RED_SUM, stream=0):
        _check(lib().dsm_group_allreduce(self.g, _dptr(d_buf, 8 * n), n, op, ctypes.c_void_p(stream)),
               "dsm_group_allreduce")

    def allreduce_counters(self, d_counters, stream=0):
        _check(lib().dsm_group_allreduce_counters(self.g, _dptr(d_counters, COUNTERS_BYTES),
                                                  ctypes.c_void_p(stream)),
               "dsm_group_allreduce_counters")

    def allreduce_aggregate(self, d_agg, stream=0):
        _check(lib().dsm_group_allreduce_aggregate(self.g, _dptr(d_agg, NAGG * 8),
                                                   ctypes.c_void_p(stream)),
               "dsm_group_allreduce_aggregate")

    def barrier(self, stream=0):
        _check(lib().dsm_group_barrier(self.g, ctypes.c_void_p(stream)), "dsm_group_barrier")

    def close(self):
        if self.g:
            lib().dsm_group_close(self.g)
            self.g = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def counters_to_dict(c):
    c = np.asarray(c, dtype=np.uint64).reshape(-1)
    return {k: int(v) for k, v in zip(COUNTER_FIELDS, c) if not k.startswith("reserved")}


def device_count():
    n = ctypes.c_int(0)
    _check(lib().dsm_device_count(ctypes.byref(n)), "dsm_device_count")
    return n.value


class Engine:
    """One dsm_ctx: np nodes per system, trace stride max_instr, bound to `device`."""

    def __init__(self, np_=8, max_instr=4096, ring_cap=0, snapshots=False, device=0, timing=False,
                 type_counts=False, issue_trace=False):
        self.np = np_
        self.max_instr = max_instr
        self.cfg = Config(np_, max_instr, ring_cap,
                          (F_SNAPSHOTS if snapshots else 0) | (F_TIMING if timing else 0) |
                          (F_TYPE_COUNTS if type_counts else 0) |
                          (F_ISSUE_TRACE if issue_trace else 0))
        self.ctx = ctypes.c_void_p()
        _check(lib().dsm_open(device, ctypes.byref(self.cfg), ctypes.byref(self.ctx)), "dsm_open")

    def close(self):
        if self.ctx:
            lib().dsm_close(self.ctx)
            self.ctx = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- host-buffer entry points ----------------------------------------------------------
    def run_packed(self, traces, counts):
        traces = np.ascontiguousarray(traces, dtype=np.uint16)
        counts = np.ascontiguousarray(counts, dtype=np.uint32)
        n = counts.shape[0]
        assert traces.shape == (n, self.np, self.max_instr), traces.shape
        assert counts.shape == (n, self.np)
        res = np.zeros(n, dtype=RESULT_DTYPE)
        cnt = np.zeros(NCOUNTERS, dtype=np.uint64)
        _check(lib().dsm_run_packed(self.ctx, _ptr(traces), _ptr(counts), n, _ptr(res), _ptr(cnt)),
               "dsm_run_packed")
        return res, counters_to_dict(cnt)

    def run_generated(self, dist, seed, n_instr, first_sys, n_sys):
        g = Gen(seed, DIST.get(dist, dist), n_instr)
        res = np.zeros(n_sys, dtype=RESULT_DTYPE)
        cnt = np.zeros(NCOUNTERS, dtype=np.uint64)
        _check(lib().dsm_run_generated(self.ctx, ctypes.byref(g), first_sys, n_sys, _ptr(res),
                                       _ptr(cnt)), "dsm_run_generated")
        return res, counters_to_dict(cnt)

    # -- device-pointer entry points (torch-owned HBM, torch streams) ----------------------
    def generate_device(self, dist, seed, n_instr, first_sys, n_sys, d_traces, d_counts, stream=0):
        g = Gen(seed, DIST.get(dist, dist), n_instr)
        _check(lib().dsm_generate_device(self.ctx, ctypes.byref(g), first_sys, n_sys,
                                         ctypes.c_void_p(d_traces), ctypes.c_void_p(d_counts),
                                         ctypes.c_void_p(stream)), "dsm_generate_device")

    def run_packed_device(self, d_traces, d_counts, n_sys, d_results, d_counters, stream=0):
        """Device pointers (ints) or tensors; a counters tensor must hold DSM_NCOUNTERS slots."""
        _check(lib().dsm_run_packed_device(self.ctx, _dptr(d_traces), _dptr(d_counts), n_sys,
                                           _dptr(d_results), _dptr(d_counters, COUNTERS_BYTES),
                                           ctypes.c_void_p(stream)), "dsm_run_packed_device")

    def run_generated_device(self, dist, seed, n_instr, first_sys, n_sys, d_results, d_counters,
                             stream=0):
        g = Gen(seed, DIST.get(dist, dist), n_instr)
        _check(lib().dsm_run_generated_device(self.ctx, ctypes.byref(g), first_sys, n_sys,
                                              _dptr(d_results), _dptr(d_counters, COUNTERS_BYTES),
                                              ctypes.c_void_p(stream)), "dsm_run_generated_device")

    def aggregate_device(self, d_results, n_sys, first_sys, d_agg, stream=0):
        """dsm_aggregate_device: per-system results -> d_agg (DSM_NAGG uint64, accumulated)."""
        _check(lib().dsm_aggregate_device(self.ctx, _dptr(d_results), n_sys, first_sys,
                                          _dptr(d_agg, NAGG * 8), ctypes.c_void_p(stream)),
               "dsm_aggregate_device")

    def node_state(self, sys, node):
        d = np.zeros(64, dtype=np.uint8)
        f = np.zeros(64, dtype=np.uint8)
        _check(lib().dsm_get_node_state(self.ctx, sys, node, _ptr(d), _ptr(f)), "dsm_get_node_state")
        return d, f

    # -- initializeProcessor's reader on the GPU ---------------------------------------------
    def parse_traces(self, files, cap):
        """files: list of bytes (core file contents, file f = node f % np of system f // np)
        -> traces [n_sys, np, max_instr] u16, counts [n_sys, np] u32, status [n_sys, np] i32"""
        n = len(files)
        assert n % self.np == 0
        text = np.frombuffer(b"".join(files) + b"\0" * 16, dtype=np.uint8)
        off = np.zeros(n + 1, dtype=np.uint64)
        off[1:] = np.cumsum([len(f) for f in files])
        tr = np.zeros((n // self.np, self.np, self.max_instr), dtype=np.uint16)
        cn = np.zeros((n // self.np, self.np), dtype=np.uint32)
        st = np.zeros((n // self.np, self.np), dtype=np.int32)
        _check(lib().dsm_parse_traces(self.ctx, _ptr(text), _ptr(off), n, cap, _ptr(tr), _ptr(cn),
                                      _ptr(st)), "dsm_parse_traces")
        return tr, cn, st

    def parse_traces_device(self, d_text, d_offsets, n_files, cap, d_traces, d_counts, d_status,
                            stream=0):
        _check(lib().dsm_parse_traces_device(self.ctx, ctypes.c_void_p(d_text),
                                             ctypes.c_void_p(d_offsets), n_files, cap,
                                             ctypes.c_void_p(d_traces), ctypes.c_void_p(d_counts),
                                             ctypes.c_void_p(d_status), ctypes.c_void_p(stream)),
               "dsm_parse_traces_device")

    def generate_text_device(self, dist, seed, n_instr, first_sys, n_sys, d_text, d_offsets,
                             stream=0):
        g = Gen(seed, DIST.get(dist, dist), n_instr)
        _check(lib().dsm_generate_text_device(self.ctx, ctypes.byref(g), first_sys, n_sys,
                                              ctypes.c_void_p(d_text), ctypes.c_void_p(d_offsets),
                                              ctypes.c_void_p(stream)), "dsm_generate_text_device")

    # -- printProcessorState on the GPU ------------------------------------------------------
    def format_dumps_device(self, d_states, n_states, d_text, d_len, state_stride=1, stream=0):
        _check(lib().dsm_format_dumps_device(self.ctx, ctypes.c_void_p(d_states), state_stride,
                                             n_states, ctypes.c_void_p(d_text),
                                             ctypes.c_void_p(d_len), ctypes.c_void_p(stream)),
               "dsm_format_dumps_device")

    def format_run_dumps_device(self, view, first_sys, n_sys, d_text, d_len, stream=0):
        _check(lib().dsm_format_run_dumps_device(self.ctx, view, first_sys, n_sys,
                                                 ctypes.c_void_p(d_text), ctypes.c_void_p(d_len),
                                                 ctypes.c_void_p(stream)),
               "dsm_format_run_dumps_device")

    def write_run_dumps(self, sys, node_mask, out_dir=None):
        _check(lib().dsm_write_run_dumps(self.ctx, sys, node_mask,
                                         out_dir.encode() if out_dir else None),
               "dsm_write_run_dumps")

    # -- schedule exploration / issue order --------------------------------------------------
    def set_schedule(self, seed, act_thresh=SCHED_LOCKSTEP):
        _check(lib().dsm_set_schedule(self.ctx, seed, act_thresh), "dsm_set_schedule")

    def issue_trace(self, sys):
        cap = self.np * self.max_instr
        ev = np.zeros(cap, dtype=np.uint32)
        n = ctypes.c_uint32(0)
        _check(lib().dsm_get_issue_trace(self.ctx, sys, _ptr(ev), cap, ctypes.byref(n)),
               "dsm_get_issue_trace")
        return ev[:min(n.value, cap)].copy()

    def last_kernel_ms(self):
        ms = ctypes.c_float(0)
        _check(lib().dsm_last_kernel_ms(self.ctx, ctypes.byref(ms)), "dsm_last_kernel_ms")
        return float(ms.value)

    def kernel_ms_history(self, cap=64):
        """Transition-kernel device times (ms) of the last min(cap, 64) runs, oldest first."""
        ms = np.zeros(max(cap, 1), dtype=np.float32)
        n = ctypes.c_uint32(0)
        _check(lib().dsm_kernel_ms_history(self.ctx, _ptr(ms), cap, ctypes.byref(n)),
               "dsm_kernel_ms_history")
        return [float(x) for x in ms[:n.value]]

    def set_budget(self, budget_log2, late_log2=9):
        _check(lib().dsm_set_budget(self.ctx, budget_log2, late_log2), "dsm_set_budget")

    def set_round_limit(self, limit_log2):
        _check(lib().dsm_set_round_limit(self.ctx, limit_log2), "dsm_set_round_limit")

    def set_inbox_limit(self, cap):
        _check(lib().dsm_set_inbox_limit(self.ctx, cap), "dsm_set_inbox_limit")

    def set_fast_forward(self, mode):
        """FF_OFF / FF_ON / FF_AUTO (dsm_set_fast_forward): only time depends on it."""
        _check(lib().dsm_set_fast_forward(self.ctx, mode), "dsm_set_fast_forward")

    def launch_info(self):
        """dsm_launch_info of the last run, plus `kernels`: the kernels that did its work
        (dsm_launch_kernel_names, e.g. "budget=sim_kernel<8, 12, 4, false, 48, 5>
        resume=ser_kernel<8, false>")."""
        li = LaunchInfo()
        _check(lib().dsm_launch_info_get(self.ctx, ctypes.byref(li)), "dsm_launch_info_get")
        d = {k: getattr(li, k) for k, _ in LaunchInfo._fields_}
        buf = ctypes.create_string_buffer(256)
        n = lib().dsm_launch_kernel_names(ctypes.byref(li), buf, 256)
        if n < 0:
            raise DsmError(n, "dsm_launch_kernel_names")
        d["kernels"] = buf.raw[:n].decode()
        return d


# -- host-only boundary helpers ------------------------------------------------------------
def parse_trace_file(path, cap=32):
    out = np.zeros(max(cap, 1), dtype=np.uint16)
    n = ctypes.c_uint32(0)
    rc = lib().dsm_parse_trace_file(path.encode(), _ptr(out), cap, ctypes.byref(n))
    _check(rc, f"dsm_parse_trace_file({path})")
    return out[:n.value].copy()


def format_dump(node, rec):
    rec = np.ascontiguousarray(rec, dtype=np.uint8)
    assert rec.size == 64
    buf = ctypes.create_string_buffer(4096)
    n = lib().dsm_format_dump(node, _ptr(rec), buf, 4096)
    if n < 0:
        raise DsmError(n, "dsm_format_dump")
    return buf.raw[:n].decode()


def split_dumps(text, lens):
    """Bulk GPU dump buffer (uint8, DUMP_SLOT bytes per record) + lengths -> list of str."""
    text = np.asarray(text, dtype=np.uint8).reshape(-1, DUMP_SLOT)
    return [bytes(text[k, :int(n)]).decode() for k, n in enumerate(np.asarray(lens))]


def format_issue_trace(events):
    events = np.ascontiguousarray(events, dtype=np.uint32)
    cap = 64 * max(len(events), 1) + 1
    buf = ctypes.create_string_buffer(cap)
    n = lib().dsm_format_issue_trace(_ptr(events), len(events), buf, cap)
    if n < 0:
        raise DsmError(n, "dsm_format_issue_trace")
    return buf.raw[:n].decode()


def node_hash(node, rec, nwords):
    rec = np.ascontiguousarray(rec, dtype=np.uint8)
    return int(lib().dsm_node_hash(node, _ptr(rec), nwords))


def pack_instr(op, addr, value=0):
    """'R'/'W' + address + value -> packed u16 (bit15 WR, bits 8-14 address, bits 0-7 value)."""
    wr = 1 if op in ("W", "WR") else 0
    return (wr << 15) | ((addr & 0x7F) << 8) | ((value & 0xFF) if wr else 0)


# -- full-size aggregates (tests/golden/aggregates.json; oracle/dsm_common.h dsm_result_digest)
_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _fmix64(z):
    z = z ^ (z >> np.uint64(33))
    z = z * np.uint64(0xff51afd7ed558ccd)
    z = z ^ (z >> np.uint64(33))
    z = z * np.uint64(0xc4ceb9fe1a85ec53)
    return z ^ (z >> np.uint64(33))


def result_digest(res, first_idx=0):
    """Sum mod 2^64 over systems of dsm_result_digest(index, result): position-sensitive, so
    it pins every system's result, not only the totals.  `res` is a RESULT_DTYPE array."""
    res = np.ascontiguousarray(res).view(RESULT_DTYPE).reshape(-1)
    with np.errstate(over="ignore"):
        idx = np.arange(first_idx, first_idx + len(res), dtype=np.uint64)
        h = _fmix64(idx * np.uint64(0x9E3779B97F4A7C15) + np.uint64(1))
        h = _fmix64(h ^ (res["status"].astype(np.uint64) | (res["rounds"].astype(np.uint64) << np.uint64(32))))
        h = _fmix64(h ^ (res["msgs"].astype(np.uint64) | (res["instrs"].astype(np.uint64) << np.uint64(32))))
        h = _fmix64(h ^ res["dump_hash"])
        h = _fmix64(h ^ res["final_hash"])
        return int(h.sum(dtype=np.uint64))


def aggregate(res, first_idx=0):
    """The golden-aggregate view of per-system results (gen_fixtures.py aggregates) of the
    systems with ids first_idx, first_idx + 1, ..."""
    res = np.ascontiguousarray(res).view(RESULT_DTYPE).reshape(-1)
    st = np.bincount((res["status"] & 0xFF).astype(np.int64), minlength=5)
    with np.errstate(over="ignore"):
        return {"systems": int(len(res)), "msgs": int(res["msgs"].sum(dtype=np.uint64)),
                "instrs": int(res["instrs"].sum(dtype=np.uint64)),
                "rounds": int(res["rounds"].sum(dtype=np.uint64)),
                "max_rounds": int(res["rounds"].max()) if len(res) else 0,
                "status": [int(x) for x in st[:5]],
                "sum_dump_hash": "0x%016x" % int(res["dump_hash"].sum(dtype=np.uint64)),
                "sum_final_hash": "0x%016x" % int(res["final_hash"].sum(dtype=np.uint64)),
                "result_digest": "0x%016x" % result_digest(res, first_idx)}


AGG_KEYS = ("systems", "msgs", "instrs", "rounds", "max_rounds", "status", "sum_dump_hash",
            "sum_final_hash", "result_digest")


def aggregate_diff(mine, gold):
    """Keys whose values differ between two aggregate dicts (empty: equal)."""
    return [k for k in AGG_KEYS if mine.get(k) != gold.get(k)]
