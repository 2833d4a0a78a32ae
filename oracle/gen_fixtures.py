#!/usr/bin/env python3
"""oracle/gen_fixtures.py -- TEST INFRASTRUCTURE ONLY: (re)generates tests/golden/.

Runs in the build container only (needs /root/reference and oracle/_ref/, built by
`make -C oracle ref`).  Everything written under tests/golden/ is DATA: inputs and expected
outputs.  Nothing written here is reference source text.

  tests/golden/inputs/<test>/core_<n>.txt      the reference's own test inputs (data files,
                                               /root/reference/tests/<test>/core_<n>.txt)
  tests/golden/lockstep/<test>/core_<n>_output.txt
                                               printProcessorState dumps produced by the
                                               reference's handler text driven under the
                                               lock-step schedule (oracle/_ref/ref_lockstep_np4_i32)
  tests/golden/lockstep/summary.json           per test: status, rounds, msgs, instrs, hashes,
                                               md5 of every dump
  tests/golden/observed/<test>.json            outcome sets of the UNMODIFIED reference binary
                                               (oracle/_ref/cache_simulator_ref, OpenMP,
                                               nondeterministic, never exits -> run under
                                               `timeout`), RUNS runs per test
  tests/golden/ensemble/<name>.npy             per-system results [n, 6] uint64 (status,
                                               rounds, msgs, instrs, dump_hash, final_hash)
                                               from oracle/_ref/ref_lockstep_np{4,8} over the
                                               counter-based generator
  tests/golden/ensemble/<name>_recs.npy        first 16 systems' dump + final node records
                                               uint8 [16, 2, np, 64]
  tests/golden/ensemble/meta.json              generator parameters per fixture
  tests/golden/lockstep/<test>/instruction_order.txt
                                               the reference's own DEBUG_INSTR issue lines
                                               (:595-598) under the lock-step schedule
                                               (oracle/_ref/ref_lockstep_np4_i32_dbg)
  tests/golden/explore/<test>.npy              per-system results [K, 6] of K seeded
                                               schedule-exploration variants (seed 7, act
                                               threshold 0x8000) of the reference's handler
                                               text (oracle/_ref/ref_lockstep_np4_i32)
  tests/golden/explore/issue_md5.json          md5 of each variant's DEBUG_INSTR issue lines
  tests/golden/dumps/random_recs.npy           4096 seeded random node records (uint8 [n, 64],
                                               every field in its valid range; record k is
                                               node k % 8)
  tests/golden/aggregates.json                 full-size aggregates of the bench workloads
                                               (python oracle/gen_fixtures.py aggregates shards
                                               types shards: + msgs_by_type per entry)
                                               (C3 1M uniform, C4 1M hot, C5 2M evict, and
                                               the 4096-system np8 fixtures): counters,
                                               status counts, hash sums and the per-system
                                               result digest (dsm_common.h), from
                                               oracle/_ref/ref_lockstep_np8 agg
  tests/golden/dumps/random_md5.json           md5 + length of the reference's OWN
                                               printProcessorState text of each of them
                                               (oracle/_ref/ref_lockstep_np8 fmt)
"""
import concurrent.futures as cf
import hashlib
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
REF = os.environ.get("REF", "/root/reference")
REFBIN = os.path.join(HERE, "_ref")
GOLD = os.path.join(REPO, "tests", "golden")
TESTS = ["sample", "test_1", "test_2", "test_3", "test_4"]
RUNS = int(os.environ.get("RUNS", "200"))

ENSEMBLES = [  # name, np, dist, seed, n_instr, first_sys, n_sys
    ("np8_uniform", 8, 0, 1, 4096, 0, 4096),
    ("np8_hot", 8, 1, 1, 4096, 0, 2048),
    ("np8_evict", 8, 2, 1, 4096, 0, 4096),
    ("np4_uniform", 4, 0, 1, 4096, 0, 4096),
    ("np8_uniform_far", 8, 0, 1, 4096, 999_000, 1024),  # ids near the end of the 1M bench set
]
RES_DT = np.dtype([("status", "<u4"), ("rounds", "<u4"), ("msgs", "<u4"), ("instrs", "<u4"),
                   ("dump_hash", "<u8"), ("final_hash", "<u8")])


def md5(b):
    return hashlib.md5(b).hexdigest()


def res_to_u64(r):
    return np.stack([r["status"].astype(np.uint64), r["rounds"].astype(np.uint64),
                     r["msgs"].astype(np.uint64), r["instrs"].astype(np.uint64),
                     r["dump_hash"], r["final_hash"]], axis=1)


def read_ref_bin(path, np_):
    rec = 32 + 2 * np_ * 64
    b = np.fromfile(path, dtype=np.uint8).reshape(-1, rec)
    res = b[:, :32].copy().view(RES_DT).reshape(-1)
    recs = b[:, 32:].reshape(-1, 2, np_, 64)
    return res, recs


def inputs():
    for t in TESTS:
        d = os.path.join(GOLD, "inputs", t)
        os.makedirs(d, exist_ok=True)
        for n in range(4):
            shutil.copyfile(os.path.join(REF, "tests", t, f"core_{n}.txt"),
                            os.path.join(d, f"core_{n}.txt"))


def lockstep():
    summary = {}
    for t in TESTS:
        with tempfile.TemporaryDirectory() as tmp:
            os.symlink(os.path.join(GOLD, "inputs"), os.path.join(tmp, "tests"))
            subprocess.run([os.path.join(REFBIN, "ref_lockstep_np4_i32"), "tests", t, "res.bin"],
                           cwd=tmp, check=True, stdout=subprocess.DEVNULL)
            res, recs = read_ref_bin(os.path.join(tmp, "res.bin"), 4)
            d = os.path.join(GOLD, "lockstep", t)
            os.makedirs(d, exist_ok=True)
            md5s = {}
            for n in range(4):
                src = os.path.join(tmp, f"core_{n}_output.txt")
                if os.path.exists(src):
                    shutil.copyfile(src, os.path.join(d, f"core_{n}_output.txt"))
                    md5s[n] = md5(open(src, "rb").read())
            r = res[0]
            summary[t] = dict(status=int(r["status"]) & 0xFF, dumped_mask=int(r["status"]) >> 8,
                              rounds=int(r["rounds"]), msgs=int(r["msgs"]),
                              instrs=int(r["instrs"]), dump_hash=int(r["dump_hash"]),
                              final_hash=int(r["final_hash"]), md5=md5s)
            np.save(os.path.join(d, "records.npy"), recs[0])
    with open(os.path.join(GOLD, "lockstep", "summary.json"), "w") as f:
        json.dump(summary, f, indent=1, sort_keys=True)


def one_run(t):
    with tempfile.TemporaryDirectory() as tmp:
        os.symlink(os.path.join(GOLD, "inputs"), os.path.join(tmp, "tests"))
        subprocess.run(["timeout", "0.3", os.path.join(REFBIN, "cache_simulator_ref"), t],
                       cwd=tmp, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        out = {}
        for n in range(4):
            p = os.path.join(tmp, f"core_{n}_output.txt")
            out[n] = open(p, "rb").read() if os.path.exists(p) else None
        return out


def observed():
    os.makedirs(os.path.join(GOLD, "observed"), exist_ok=True)
    with cf.ThreadPoolExecutor(8) as ex:
        for t in TESTS:
            runs = list(ex.map(one_run, [t] * RUNS))
            cores = {}
            for n in range(4):
                outs, missing = {}, 0
                for r in runs:
                    b = r[n]
                    if b is None or len(b) == 0:
                        missing += 1
                        continue
                    h = md5(b)
                    e = outs.setdefault(h, {"count": 0, "text": b.decode()})
                    e["count"] += 1
                cores[str(n)] = {"missing": missing, "outcomes": outs}
            with open(os.path.join(GOLD, "observed", f"{t}.json"), "w") as f:
                json.dump({"runs": RUNS, "binary": "assignment.c, gcc -O2 -fopenmp, timeout 0.3 s",
                           "cores": cores}, f, indent=1, sort_keys=True)


def ensemble():
    d = os.path.join(GOLD, "ensemble")
    os.makedirs(d, exist_ok=True)
    meta = {}
    for name, np_, dist, seed, n_instr, first, n in ENSEMBLES:
        with tempfile.TemporaryDirectory() as tmp:
            out = os.path.join(tmp, "e.bin")
            subprocess.run([os.path.join(REFBIN, f"ref_lockstep_np{np_}"), "gen", str(dist),
                            str(seed), str(n_instr), str(first), str(n), out], check=True)
            res, recs = read_ref_bin(out, np_)
        np.save(os.path.join(d, f"{name}.npy"), res_to_u64(res))
        np.save(os.path.join(d, f"{name}_recs.npy"), np.ascontiguousarray(recs[:16]))
        meta[name] = dict(np=np_, dist=dist, seed=seed, n_instr=n_instr, first_sys=first, n_sys=n)
    with open(os.path.join(d, "meta.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)


# name: dist, seed, n_instr, first_sys, n_sys -- bench.py's CONFIGS at N=1 (rank 0's shard),
# plus the 4096-system fixtures (pins the numpy digest against np8_*.npy)
AGGREGATES = {
    "random": (0, 1, 4096, 0, 1 << 20),
    "hot": (1, 1, 4096, 0, 1 << 20),
    "evict": (2, 1, 4096, 0, 2 << 20),
    "np8_uniform": (0, 1, 4096, 0, 4096),
    "np8_hot": (1, 1, 4096, 0, 2048),
    "np8_evict": (2, 1, 4096, 0, 4096),
}


def aggregates():
    """Full-size golden aggregates: the reference's own handler text (ref_lockstep_np8 agg,
    lock-step schedule) over every system of each bench workload, in forked slices."""
    p = os.path.join(GOLD, "aggregates.json")
    out = json.load(open(p)) if os.path.exists(p) else {}
    only = os.environ.get("AGG_ONLY")
    for name, (dist, seed, n_instr, first, n) in AGGREGATES.items():
        if only and name not in only.split(","):
            continue
        r = subprocess.run([os.path.join(REFBIN, "ref_lockstep_np8"), "agg", str(dist), str(seed),
                            str(n_instr), str(first), str(n), str(os.cpu_count() or 8)],
                           check=True, capture_output=True, text=True)
        d = json.loads(r.stdout.strip().splitlines()[-1])
        d.update(np=8, dist=dist, seed=seed, n_instr=n_instr, first_sys=first,
                 producer="oracle/_ref/ref_lockstep_np8 agg (assignment.c handler/issue text, "
                          "lock-step schedule)")
        out[name] = d
        print("  ", name, d["msgs"], d["result_digest"], flush=True)
        with open(p, "w") as f:
            json.dump(out, f, indent=1, sort_keys=True)


# multi-GPU bench (weak scaling, bench.shard): rank r simulates ids [r*n, (r+1)*n).  Every
# shard of an 8-GPU run gets its own reference aggregate ("<config>@<r>"; shard 0 is the
# "<config>" entry above), and the job totals at 2, 4 and 8 GPUs ("<config>@x<N>") are the
# merge of shards 0..N-1 -- sums mod 2^64 for the hashes and the position-sensitive digest,
# max for max_rounds -- which equals one reference run over ids [0, N*n)
# (tests/test_aggregates.py checks that identity on small ranges).
SHARDED = {"random": 0, "hot": 1, "evict": 2}
MAX_RANKS = 8
M64 = (1 << 64) - 1


def merge_aggregates(parts):
    """The aggregate of a union of disjoint system ranges (ref_lockstep.c agg_merge)."""
    out = dict(systems=0, msgs=0, instrs=0, rounds=0, max_rounds=0, status=[0] * 5)
    h = dict(sum_dump_hash=0, sum_final_hash=0, result_digest=0)
    for p in parts:
        for k in ("systems", "msgs", "instrs", "rounds"):
            out[k] += p[k]
        out["max_rounds"] = max(out["max_rounds"], p["max_rounds"])
        out["status"] = [a + b for a, b in zip(out["status"], p["status"])]
        for k in h:
            h[k] = (h[k] + int(p[k], 16)) & M64
    out.update({k: "0x%016x" % v for k, v in h.items()})
    if all("msgs_by_type" in p for p in parts):
        out["msgs_by_type"] = [sum(x) for x in zip(*(p["msgs_by_type"] for p in parts))]
    return out


def types():
    """Handled messages per transactionType (assignment.c:20-34) of every reference
    aggregate entry (ref_lockstep agg's msgs_by_type), added to the entries that lack them;
    the re-run must reproduce every other field of the entry.  The 2/4/8-GPU job totals are
    the shard sums (shards() after this)."""
    p = os.path.join(GOLD, "aggregates.json")
    out = json.load(open(p))
    only = os.environ.get("AGG_ONLY")
    for key, d in sorted(out.items()):
        if "@x" in key or "msgs_by_type" in d or (only and key.split("@")[0] not in only.split(",")):
            continue
        res = subprocess.run([os.path.join(REFBIN, "ref_lockstep_np8"), "agg", str(d["dist"]),
                              str(d["seed"]), str(d["n_instr"]), str(d["first_sys"]),
                              str(d["systems"]), str(os.cpu_count() or 8)],
                             check=True, capture_output=True, text=True)
        r = json.loads(res.stdout.strip().splitlines()[-1])
        for k in ("systems", "msgs", "instrs", "rounds", "max_rounds", "status", "sum_dump_hash",
                  "sum_final_hash", "result_digest"):
            assert r[k] == d[k], (key, k, r[k], d[k])
        assert sum(r["msgs_by_type"]) == d["msgs"], key
        d["msgs_by_type"] = r["msgs_by_type"]
        print("  ", key, r["msgs_by_type"], flush=True)
        with open(p, "w") as f:
            json.dump(out, f, indent=1, sort_keys=True)


def shards():
    """Reference aggregates of shards 1..7 of every bench workload (shard 0 is aggregates()'s
    entry) and the 2/4/8-GPU job totals."""
    p = os.path.join(GOLD, "aggregates.json")
    out = json.load(open(p))
    only = os.environ.get("AGG_ONLY")
    for name, dist in SHARDED.items():
        if only and name not in only.split(","):
            continue
        base = out[name]
        n, seed, n_instr = base["systems"], base["seed"], base["n_instr"]
        parts = [base]
        for r in range(1, MAX_RANKS):
            key = f"{name}@{r}"
            d = out.get(key)
            if d is None or d.get("first_sys") != r * n or d.get("systems") != n:
                res = subprocess.run([os.path.join(REFBIN, "ref_lockstep_np8"), "agg", str(dist),
                                      str(seed), str(n_instr), str(r * n), str(n),
                                      str(os.cpu_count() or 8)],
                                     check=True, capture_output=True, text=True)
                d = json.loads(res.stdout.strip().splitlines()[-1])
                d.update(np=8, dist=dist, seed=seed, n_instr=n_instr, first_sys=r * n,
                         producer="oracle/_ref/ref_lockstep_np8 agg (assignment.c handler/issue "
                                  "text, lock-step schedule)")
                out[key] = d
                print("  ", key, d["msgs"], d["result_digest"], flush=True)
                with open(p, "w") as f:
                    json.dump(out, f, indent=1, sort_keys=True)
            parts.append(d)
        for g in (2, 4, 8):
            t = merge_aggregates(parts[:g])
            t.update(np=8, dist=dist, seed=seed, n_instr=n_instr, first_sys=0, gpus=g,
                     producer=f"merge of the reference aggregates of shards 0..{g - 1} "
                              f"(oracle/gen_fixtures.py shards)")
            out[f"{name}@x{g}"] = t
        with open(p, "w") as f:
            json.dump(out, f, indent=1, sort_keys=True)


EXPLORE_K, EXPLORE_SEED, EXPLORE_THRESH = 256, 7, 0x8000
ISSUE_RE = re.compile(rb"^Processor \d+: instr type=.*\n", re.M)


def explore():
    d = os.path.join(GOLD, "explore")
    os.makedirs(d, exist_ok=True)
    issue = {}
    for t in TESTS:
        with tempfile.TemporaryDirectory() as tmp:
            os.symlink(os.path.join(GOLD, "inputs"), os.path.join(tmp, "tests"))
            dbg = os.path.join(REFBIN, "ref_lockstep_np4_i32_dbg")
            out = subprocess.run([dbg, "tests", t, "res.bin"], cwd=tmp, check=True,
                                 capture_output=True).stdout
            with open(os.path.join(GOLD, "lockstep", t, "instruction_order.txt"), "wb") as f:
                f.write(b"".join(ISSUE_RE.findall(out)))
            args = [t, "res.bin", str(EXPLORE_SEED), hex(EXPLORE_THRESH), "0", str(EXPLORE_K)]
            subprocess.run([os.path.join(REFBIN, "ref_lockstep_np4_i32"), "tests"] + args,
                           cwd=tmp, check=True, stdout=subprocess.DEVNULL)
            res, _ = read_ref_bin(os.path.join(tmp, "res.bin"), 4)
            np.save(os.path.join(d, f"{t}.npy"), res_to_u64(res))
            out = subprocess.run([dbg, "tests"] + args, cwd=tmp, check=True,
                                 capture_output=True).stdout
            lines = ISSUE_RE.findall(out)
            k, md5s = 0, []
            for r in res:
                md5s.append(md5(b"".join(lines[k:k + int(r["instrs"])])))
                k += int(r["instrs"])
            assert k == len(lines)
            issue[t] = md5s
    with open(os.path.join(d, "issue_md5.json"), "w") as f:
        json.dump({"k": EXPLORE_K, "seed": EXPLORE_SEED, "thresh": EXPLORE_THRESH,
                   "issue_md5": issue}, f, indent=0)


def random_records(n, seed):
    """Node records with every field in its valid range; cache states uniform over the four
    (so about a quarter of the cache lines print the 9-character "EXCLUSIVE")."""
    rng = np.random.default_rng(seed)
    r = np.zeros((n, 64), dtype=np.uint8)
    r[:, 0:16] = rng.integers(0, 256, (n, 16))          # memory
    r[:, 16:32] = rng.integers(0, 256, (n, 16))         # directory bitVector
    r[:, 32:48] = rng.integers(0, 3, (n, 16))           # directory state EM/S/U
    r[:, 48:52] = rng.integers(0, 256, (n, 4))          # cache address
    r[:, 52:56] = rng.integers(0, 256, (n, 4))          # cache value
    r[:, 56:60] = rng.integers(0, 4, (n, 4))            # cache state
    r[:, 60] = rng.integers(0, 256, n)                  # pendingWriteValue (not printed)
    return r


def dumps():
    d = os.path.join(GOLD, "dumps")
    os.makedirs(d, exist_ok=True)
    recs = random_records(4096, 20261016)
    with tempfile.TemporaryDirectory() as tmp:
        rin, rout = os.path.join(tmp, "r.bin"), os.path.join(tmp, "t.bin")
        recs.tofile(rin)
        subprocess.run([os.path.join(REFBIN, "ref_lockstep_np8"), "fmt", rin, rout], check=True)
        blob = open(rout, "rb").read()
    out, off = [], 0
    while off < len(blob):
        n = int.from_bytes(blob[off:off + 4], "little")
        out.append(dict(len=n, md5=md5(blob[off + 4:off + 4 + n])))
        off += 4 + n
    assert len(out) == len(recs)
    np.save(os.path.join(d, "random_recs.npy"), recs)
    with open(os.path.join(d, "random_md5.json"), "w") as f:
        json.dump({"producer": "oracle/_ref/ref_lockstep_np8 fmt (assignment.c:824-876)",
                   "np": 8, "texts": out}, f, indent=0)


if __name__ == "__main__":
    if not os.path.exists(os.path.join(REF, "assignment.c")) or \
            not os.path.exists(os.path.join(REFBIN, "ref_lockstep_np8")):
        sys.exit("gen_fixtures: needs /root/reference and oracle/_ref (make -C oracle ref)")
    steps = sys.argv[1:] or ["inputs", "lockstep", "observed", "ensemble", "dumps", "explore"]
    for s in steps:
        print("gen_fixtures:", s, flush=True)
        globals()[s]()
