#!/usr/bin/env python3
"""bench.py -- simulated coherence transactions/sec (whole node) + % HBM roofline.

A "step" is one pass of the hot path (lock-step transition kernel + 256-deep re-run of
overflowing systems + counter reduction) over this rank's batch of synthetic systems, whose
packed traces are already resident in HBM (generated on the device before warmup; the
generator pass is timed separately as the trace-streaming phase).

Default workload (N=1): BASELINE.json configs[2] / SURVEY 8d C3 -- 1M synthetic 8-node
systems, uniform RD/WR over 0x00-0x7F, 4096 instructions per node, seed 1.  With N GPUs each
rank simulates its own 1M systems (ids rank*1M ..), i.e. weak scaling; the only collective is
the final RCCL all-reduce of the counters.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config random|hot|evict]
    torchrun --nproc-per-node N bench.py --gpus N ...

With --gpus N > 1 and no torch.distributed launcher around it (WORLD_SIZE unset), the process
starts N fresh rank processes itself (before anything touches the GPU), relays rank 0's JSON
line and fails if any rank fails.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "hp-assignment-2_amd")
ORACLE = os.path.join(REPO, "oracle")
if PKG not in sys.path:
    sys.path.insert(0, PKG)

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
METRIC = "simulated coherence transactions/sec (whole node) + % HBM roofline, 1/2/4/8 GPU"
UNIT = "transactions/s"

CONFIGS = {
    # name: (dist, systems per GPU, instructions per node, seed, workload description)
    "random": ("uniform", 1 << 20, 4096, 1,
               "C3: 1M synthetic 8-node systems/GPU, uniform RD/WR over 0x00-0x7F, 4096 instr/core"),
    "hot": ("hot", 1 << 20, 4096, 1,
            "C4: 1M hot-line 8-node systems/GPU, RD/WR over {0x00,0x11,0x22,0x33}, 4096 instr/core"),
    "evict": ("evict", 2 << 20, 4096, 1,
              "C5: 2M eviction-heavy 8-node systems/GPU (16M on 8), {a: a%4==0}, 4096 instr/core"),
}
NP = 8


def shard(rank, n_per_rank):
    """System ids simulated by `rank` (weak scaling: a fixed n_per_rank per GPU)."""
    return rank * n_per_rank, n_per_rank


def reduce_counters(vec, dist_mod=None):
    """All-reduce a dsm_counters vector (DSM_NCOUNTERS uint64) across ranks: sums (mod 2^64) for every
    slot except max_rounds (slot 24), which is a max.  `vec` is a torch int64 tensor."""
    return reduce_vector(vec, dist_mod, (24,))


def launch_ranks(n, argv, cmd=None, timeout=None):
    """Start n rank processes of this script (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR /
    MASTER_PORT set; one GPU each by LOCAL_RANK) and wait for them.  Rank 0's stdout is
    inherited (its JSON line is the result); the others' stdout is discarded.  When a rank
    fails, the rest are terminated (by the PIDs started here) and its exit code returned.
    `cmd` replaces [python, bench.py] (tests)."""
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    base = cmd or [sys.executable, os.path.abspath(__file__)]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen(base + list(argv), env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    rc = 0
    deadline = None if timeout is None else time.time() + timeout
    pending = list(procs)
    while pending:
        for p in list(pending):
            code = p.poll()
            if code is None:
                continue
            pending.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 1
                for q in pending:
                    q.terminate()
        if deadline is not None and time.time() > deadline and pending:
            for q in pending:
                q.kill()
            rc = rc or 124
        time.sleep(0.05)
    return rc


def cgroup_cpus():
    """CPUs this job may use by its cgroup's CPU quota (cpu.max, cgroup v2; cfs quota, v1),
    or None when unlimited / unreadable."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
        if q != "max":
            return float(q) / float(p)
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            p = int(f.read())
        if q > 0:
            return q / p
    except (OSError, ValueError):
        pass
    return None


def host_cpu():
    """The host's CPU as the baseline uses it.  The baseline runs on the job's CPU share: the
    GPU pool gives a one-GPU job 16 CPUs and sets OMP_NUM_THREADS to it (os.cpu_count() shows
    the whole machine's); the threads used are OMP_NUM_THREADS, else the CPUs this process may
    run on, capped by the cgroup quota."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS", "")
    quota = cgroup_cpus()
    threads = int(omp) if omp.isdigit() and int(omp) > 0 else aff
    if quota is not None:
        threads = min(threads, max(1, int(quota)))
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return dict(threads=min(threads, aff), nproc=os.cpu_count(), affinity=aff, model=model,
                omp_num_threads=omp or None, cgroup_cpus=quota)


def cpu_baseline(dist, n_instr, seed, n_sample, threads):
    """The CPU oracle (clean-room C restatement, gcc -O2 -fopenmp, OpenMP over systems) on a
    bounded sample of the same system ids -- a reported baseline, not the target."""
    if ORACLE not in sys.path:
        sys.path.insert(0, ORACLE)
    import pyoracle
    pyoracle.lib()
    t0 = time.perf_counter()
    res, _ = pyoracle.run_generated(NP, dist, seed, n_instr, 0, n_sample, nthreads=threads)
    dt = time.perf_counter() - t0
    msgs = int(res["msgs"].sum())
    return res, dict(value=msgs / dt, unit=UNIT, cores=threads, kind="port",
                     sample=f"systems 0..{n_sample - 1} of the same workload ({msgs} transactions,"
                            f" {dt:.2f} s wall, {threads} OpenMP threads, traces generated lazily)",
                     msgs=msgs, instrs=int(res["instrs"].sum()))


def cpu_baseline_reference(dist, n_instr, seed, n_sample, procs):
    """The REFERENCE's own transition code (assignment.c handler + issue text, compiled
    gcc -O2 from /root/reference by oracle/build_ref.sh into oracle/_ref/, driven under the
    same lock-step schedule) over systems 0..n_sample-1 of the same workload, in `procs`
    forked processes.  Timed: run_system only (trace generation + initializeProcessor
    excluded, as the GPU's timed region starts with traces in HBM); rate = transactions /
    the slowest process's simulation time.  None when oracle/_ref was not built."""
    exe = os.path.join(ORACLE, "_ref", f"ref_lockstep_np{NP}")
    if not os.path.exists(exe):
        return None
    import subprocess
    dcode = {"uniform": 0, "hot": 1, "evict": 2}[dist]
    r = subprocess.run([exe, "bench", str(dcode), str(seed), str(n_instr), "0", str(n_sample),
                        str(procs)], capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        return None
    d = json.loads(r.stdout.strip().splitlines()[-1])
    t = d["sim_ns_max"] * 1e-9
    return dict(value=d["msgs"] / t, unit=UNIT, cores=procs, kind="reference", msgs=d["msgs"],
                sample=f"systems 0..{n_sample - 1} of the same workload ({d['msgs']} transactions); "
                       f"assignment.c's own handler/issue code (gcc -O2) under the lock-step "
                       f"schedule, {procs} processes, simulation time of the slowest "
                       f"{t:.2f} s (generation and initializeProcessor untimed)")


DIST_CODE = {"uniform": 0, "hot": 1, "evict": 2}
GOLDEN = os.path.join(REPO, "tests", "golden")
# the aggregate of a system range as a vector (all-reduced across ranks: sums mod 2^64, a max
# for max_rounds) followed by the per-rank shard verdicts (ranks whose shard equals its
# reference aggregate / differs / has none)
AGG_VEC = ("systems", "msgs", "instrs", "rounds", "max_rounds", "st0", "st1", "st2", "st3", "st4",
           "sum_dump_hash", "sum_final_hash", "result_digest", "shards_ok", "shards_bad",
           "shards_unpinned")
AGG_MAX = AGG_VEC.index("max_rounds")


def _load_json(p):
    try:
        with open(p) as f:
            return json.load(f)
    except (OSError, ValueError):
        return {}


def golden_for(dname, seed, n_instr, first, n):
    """The reference's aggregate of system ids [first, first + n) of a workload and where it
    comes from: an entry of tests/golden/aggregates.json over exactly that range (the
    reference's handler text over every system -- oracle/gen_fixtures.py aggregates / shards:
    each shard of the 1..8-GPU bench and the job totals at 2/4/8 GPUs), else the aggregate of
    the slice of a golden per-system fixture (tests/golden/ensemble/np8_*.npy) that holds the
    range.  (None, None) when nothing pins it."""
    import pydsm
    code = DIST_CODE[dname]
    want = dict(np=NP, dist=code, seed=seed, n_instr=n_instr)
    for key, g in sorted(_load_json(os.path.join(GOLDEN, "aggregates.json")).items()):
        if all(g.get(k) == v for k, v in want.items()) and g.get("first_sys") == first \
                and g.get("systems") == n:
            return g, "aggregates.json:" + key
    for key, m in sorted(_load_json(os.path.join(GOLDEN, "ensemble", "meta.json")).items()):
        if all(m.get(k) == v for k, v in want.items()) and \
                m["first_sys"] <= first and first + n <= m["first_sys"] + m["n_sys"]:
            lo = first - m["first_sys"]
            g = np.load(os.path.join(GOLDEN, "ensemble", key + ".npy"))[lo:lo + n]
            res = np.zeros(n, dtype=pydsm.RESULT_DTYPE)
            for i, f in enumerate(("status", "rounds", "msgs", "instrs", "dump_hash",
                                   "final_hash")):
                res[f] = g[:, i]
            return pydsm.aggregate(res, first), f"ensemble/{key}.npy[{lo}:{lo + n}]"
    return None, None


def agg_to_vec(a, verdict=None):
    """An aggregate dict (+ this rank's shard verdict: 'ok' / 'bad' / 'unpinned') as AGG_VEC."""
    v = [a["systems"], a["msgs"], a["instrs"], a["rounds"], a["max_rounds"]] + list(a["status"]) + \
        [int(a[k], 16) for k in ("sum_dump_hash", "sum_final_hash", "result_digest")] + \
        [int(verdict == "ok"), int(verdict == "bad"), int(verdict == "unpinned")]
    return np.array([x & 0xFFFFFFFFFFFFFFFF for x in v], dtype=np.uint64)


def vec_to_agg(v):
    v = [int(x) for x in np.asarray(v, dtype=np.uint64)]
    a = dict(zip(AGG_VEC, v))
    out = {k: a[k] for k in ("systems", "msgs", "instrs", "rounds", "max_rounds")}
    out["status"] = [a[f"st{i}"] for i in range(5)]
    out.update({k: "0x%016x" % a[k] for k in ("sum_dump_hash", "sum_final_hash", "result_digest")})
    return out, dict(ok=a["shards_ok"], bad=a["shards_bad"], unpinned=a["shards_unpinned"])


def reduce_vector(vec, dist_mod, max_slots=()):
    """All-reduce an int64 torch vector across ranks: sums (mod 2^64) except the `max_slots`."""
    if dist_mod is None or not dist_mod.is_initialized():
        return vec
    mx = [vec[i:i + 1].clone() for i in max_slots]
    dist_mod.all_reduce(vec, op=dist_mod.ReduceOp.SUM)
    for i, m in zip(max_slots, mx):
        dist_mod.all_reduce(m, op=dist_mod.ReduceOp.MAX)
        vec[i:i + 1] = m
    return vec


def check_aggregate(mine, gold, counters=None):
    """Differences between an aggregate (and the engine's own counters over the same systems,
    when given) and the reference's; [] when equal."""
    import pydsm
    diff = pydsm.aggregate_diff(mine, gold)
    if counters is not None:
        for k in ("msgs", "instrs", "rounds", "systems", "max_rounds"):
            if counters[k] != gold[k] and k not in diff:
                diff.append("counter " + k)
        if counters["sum_final_hash"] != int(gold["sum_final_hash"], 16):
            diff.append("counter sum_final_hash")
    return diff


def shard_parity(dname, seed, n_instr, first, res_host, counters):
    """This rank's shard against the reference: ('ok' | 'bad' | 'unpinned', message)."""
    import pydsm
    mine = pydsm.aggregate(res_host, first)
    gold, src = golden_for(dname, seed, n_instr, first, len(res_host))
    if gold is None:
        return mine, "unpinned", f"shard [{first}, {first + len(res_host)}): no reference aggregate"
    diff = check_aggregate(mine, gold, counters)
    return mine, ("bad" if diff else "ok"), (
        f"shard [{first}, {first + len(res_host)}) " +
        (f"== reference ({src})" if not diff else f"MISMATCH vs {src}: " + ",".join(diff)))


def job_parity(dname, seed, n_instr, world, n_per_rank, total_vec, counters):
    """The job's all-reduced aggregate and counters (ids [0, world * n_per_rank)) against the
    reference, plus the per-shard tally: the bench line's `parity` string."""
    tot, tally = vec_to_agg(total_vec)
    gold, src = golden_for(dname, seed, n_instr, 0, world * n_per_rank)
    if gold is None:
        job = f"job total over {world} shard(s) unpinned (no reference aggregate for " \
              f"[0, {world * n_per_rank}))"
    else:
        diff = check_aggregate(tot, gold, counters)
        job = (f"full-size aggregate == reference (job total over {world} shard(s), {src})"
               if not diff else f"AGGREGATE MISMATCH vs {src}: " + ",".join(diff))
    shards = f"{tally['ok']}/{world} shards == their reference aggregates"
    if tally["bad"]:
        shards += f"; {tally['bad']} SHARD MISMATCH"
    if tally["unpinned"]:
        shards += f"; {tally['unpinned']} unpinned"
    return job + "; " + shards, dict(job_source=src, shards=tally)


def traffic_from_profiles(config):
    p = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        with open(p) as f:
            d = json.load(f)
        e = d.get(config)
        return e if e else None
    except (OSError, ValueError):
        return None


def issue_from_profiles(config):
    """Per transition kernel: VALU-busy fraction, waves per SIMD, wait / issue-stall fractions,
    LDS bank conflicts (profiles/pmc_issue.json, tools/issue.py), or None."""
    return _load_json(os.path.join(REPO, "profiles", "pmc_issue.json")).get(config) or None


def run_c_driver(args):
    """bench.py --driver c: the C multi-GPU driver (hp-assignment-2_amd/dsm_ensemble: one
    process, one host thread per GPU, RCCL all-reduce through dsm_group_*) over N GPUs; its
    per-rank aggregates, job total, counters and per-type counts are checked here against the
    reference's, and the bench line is printed from its JSON.  Returns the exit code (3 on a
    parity mismatch)."""
    import pydsm
    dname, n_sys, n_instr, seed, workload = CONFIGS[args.config]
    if args.systems:
        n_sys = args.systems
    cmd = [os.path.join(PKG, "dsm_ensemble"), "--gpus", str(args.gpus), "--config", args.config,
           "--steps", str(args.steps), "--warmup", str(args.warmup), "--systems", str(n_sys)]
    if not args.no_types:
        cmd.append("--type-counts")
    r = subprocess.run(cmd, capture_output=True, text=True)
    sys.stderr.write(r.stderr)
    if r.returncode != 0:
        return r.returncode
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    tally = dict(ok=0, bad=0, unpinned=0)
    for rk in d["ranks"]:
        gold, src = golden_for(dname, seed, n_instr, rk["first_sys"], rk["systems"])
        if gold is None:
            tally["unpinned"] += 1
            continue
        diff = pydsm.aggregate_diff(rk["aggregate"], gold)
        tally["bad" if diff else "ok"] += 1
        print(f"bench.py --driver c: rank {rk['rank']} shard [{rk['first_sys']}, "
              f"{rk['first_sys'] + rk['systems']}) " +
              (f"== reference ({src})" if not diff else f"MISMATCH vs {src}: " + ",".join(diff)),
              file=sys.stderr, flush=True)
    world = d["n_gpus"]
    counters = dict(d["counters"], sum_final_hash=int(d["counters"]["sum_final_hash"], 16))
    gold, src = golden_for(dname, seed, n_instr, 0, world * n_sys)
    if gold is None:
        parity = f"job total over {world} shard(s) unpinned"
    else:
        diff = check_aggregate(d["total"], gold, counters)
        parity = (f"full-size aggregate == reference (job total over {world} shard(s), {src})"
                  if not diff else f"AGGREGATE MISMATCH vs {src}: " + ",".join(diff))
    parity += f"; {tally['ok']}/{world} shards == their reference aggregates"
    if tally["bad"]:
        parity += f"; {tally['bad']} SHARD MISMATCH"
    by_type = d.get("msgs_by_type")
    if by_type is not None:
        if sum(by_type) != counters["msgs"] or d.get("type_pass_msgs") != counters["msgs"]:
            parity += "; MSGS_BY_TYPE MISMATCH (sum != messages)"
        elif gold is not None and gold.get("msgs_by_type"):
            parity += ("; msgs_by_type == reference (13 types)" if by_type == gold["msgs_by_type"]
                       else "; MSGS_BY_TYPE MISMATCH vs reference")
    kavg = float(np.mean(d["kernel_ms"])) if d["kernel_ms"] else float("nan")
    r0 = d["ranks"][0]["aggregate"]
    alg_bytes = 2 * r0["instrs"] + (32 + 4 * NP) * r0["systems"]
    ach = alg_bytes / (kavg * 1e-3) / 1e9
    tr = traffic_from_profiles(args.config) or {}
    traffic = None
    if tr.get("sim_kernel") and tr.get("ser_kernel"):
        traffic = int(tr["sim_kernel"]["bytes_per_launch"] + tr["ser_kernel"]["bytes_per_launch"])
    rec = {
        "metric": METRIC, "value": d["value"], "unit": UNIT, "n_gpus": world,
        "steps": d["steps"], "warmup": d["warmup"], "ms_per_step": d["ms_per_step"],
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (counter-based generator, seed %d)" % seed,
        "config": {"workload": workload, "systems_per_gpu": n_sys, "np": NP,
                   "instr_per_node": n_instr, "dist": dname,
                   "parallelism": f"ensemble-dp{world} (C driver: one host thread per GPU)",
                   "traces": "packed u16 traces resident in HBM"},
        "roofline": dict(bound="hbm", achieved=round(ach, 2), peak=HBM_PEAK_GBS, unit="GB/s",
                         frac=round(ach / HBM_PEAK_GBS, 6), traffic=traffic,
                         kernel_ms_avg=round(kavg, 3), algorithmic_bytes_per_launch=alg_bytes,
                         per_unit="2 B per consumed packed instruction + 32 B result + 4*np B "
                                  "counts per system; 'launch' = one step's budget + resume launches"),
        "cpu_baseline": None,
        "driver": d["driver"],
        "collective": d["collective"],
        "counters": d["counters"],
        "msgs_by_type": dict(zip(pydsm.TYPE_NAMES, by_type)) if by_type is not None else None,
        "kernel_ms": d["kernel_ms"],
        "parity": parity,
        "parity_detail": dict(job_source=src, shards=tally),
    }
    print(json.dumps(rec), flush=True)
    return 3 if "MISMATCH" in parity else 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="random", choices=sorted(CONFIGS))
    ap.add_argument("--systems", type=int, default=0, help="override systems per GPU")
    ap.add_argument("--ring", type=int, default=0)
    ap.add_argument("--fused", action="store_true",
                    help="generate instructions inside the transition kernel (no HBM traces)")
    ap.add_argument("--cpu-sample", type=int, default=0,
                    help="systems for the port baseline (0: the whole workload)")
    ap.add_argument("--cpu-ref-sample", type=int, default=0,
                    help="systems for the reference baseline (0: the whole workload)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-dump", action="store_true", help="skip the GPU dump-formatter phase")
    ap.add_argument("--parse-systems", type=int, default=65536,
                    help="systems whose core files are generated as text and GPU-parsed (0: skip)")
    ap.add_argument("--no-types", action="store_true",
                    help="skip the per-type message count pass (parity only, after timing)")
    ap.add_argument("--driver", default="py", choices=("py", "c"),
                    help="c: the C multi-GPU driver (hp-assignment-2_amd/dsm_ensemble: one host "
                         "thread per GPU, RCCL), checked here against the reference aggregates")
    args = ap.parse_args()

    if args.driver == "c":
        if "WORLD_SIZE" in os.environ and os.environ["WORLD_SIZE"] != "1":
            raise SystemExit("bench.py --driver c runs every GPU from one process: launch it "
                             "without torchrun")
        sys.exit(run_c_driver(args))
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one fresh process per GPU, started before this process touches the GPU
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))

    import torch
    import torch.distributed as dist
    import pydsm

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and not (world == 1 and args.gpus <= 1):
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    # test knobs (tests/test_gpu_bench.py): every rank on one device, gloo for the counters
    if os.environ.get("DSM_BENCH_DEVICE"):
        local = int(os.environ["DSM_BENCH_DEVICE"])
    # nccl (default): the collectives are RCCL over xGMI issued by libdsm itself (dsm_group_*,
    # one communicator per GPU, even at one rank); torch.distributed (gloo, CPU) only hands
    # rank 0's RCCL id to the other ranks.  gloo (tests: several ranks on one GPU, which RCCL
    # refuses): the collectives through a torch.distributed gloo group on host tensors.
    backend = os.environ.get("DSM_BENCH_BACKEND", "nccl")
    use_group = backend == "nccl"
    use_dist = world > 1 or (not use_group and os.environ.get("DSM_BENCH_DIST") == "1")
    torch.cuda.set_device(local)
    if use_dist:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo")
    group = None
    if use_group:
        uid = [pydsm.Group.unique_id() if rank == 0 else None]
        if use_dist:
            dist.broadcast_object_list(uid, src=0)
        group = pydsm.Group(local, world, rank, uid[0])

    dname, n_sys, n_instr, seed, workload = CONFIGS[args.config]
    if args.systems:
        n_sys = args.systems
    first, n_sys = shard(rank, n_sys)
    dev = torch.device("cuda", local)
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream

    eng = pydsm.Engine(NP, n_instr, ring_cap=args.ring, device=local, timing=True)
    cnt = torch.zeros(pydsm.NCOUNTERS, dtype=torch.int64, device=dev)
    out = torch.empty((n_sys, 4), dtype=torch.int64, device=dev)

    trace_stream = None
    if not args.fused:
        traces = torch.empty((n_sys, NP, n_instr), dtype=torch.int16, device=dev)
        counts = torch.empty((n_sys, NP), dtype=torch.int32, device=dev)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        eng.generate_device(dname, seed, n_instr, first, n_sys, traces.data_ptr(),
                            counts.data_ptr(), sp)              # cold (first-touch) pass
        ev0.record(stream)
        eng.generate_device(dname, seed, n_instr, first, n_sys, traces.data_ptr(),
                            counts.data_ptr(), sp)
        ev1.record(stream)
        torch.cuda.synchronize(dev)
        gms = ev0.elapsed_time(ev1)
        gbytes = traces.numel() * 2 + counts.numel() * 4
        trace_stream = dict(kernel="gen_kernel (trace generator, writes packed traces)",
                            bytes=gbytes, ms=round(gms, 3),
                            achieved_gbs=round(gbytes / gms / 1e6, 1), peak_gbs=HBM_PEAK_GBS,
                            frac=round(gbytes / gms / 1e6 / HBM_PEAK_GBS, 4))

    def step():
        cnt.zero_()
        if args.fused:
            eng.run_generated_device(dname, seed, n_instr, first, n_sys, out.data_ptr(),
                                     cnt.data_ptr(), sp)
        else:
            eng.run_packed_device(traces, counts, n_sys, out, cnt, sp)

    def barrier():
        if group is not None:
            group.barrier(sp)           # RCCL all-reduce of one word, then a stream wait
        elif use_dist:
            dist.barrier()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)

    barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()          # asynchronous: the steps queue back to back on the stream
    torch.cuda.synchronize(dev)
    barrier()
    elapsed = time.perf_counter() - t0
    # the transition kernel's device time per step (HIP events around its launches, on the
    # stream they run on), read after the timed region
    kms = eng.kernel_ms_history(min(args.steps, 64))

    # initializeProcessor's reader on the GPU (parse_kernel): the same workload's core files as
    # text (shipped-test format) for the first --parse-systems systems, scanned back into packed
    # traces; timed separately, not part of `value`; checked bit-exact against gen_kernel
    trace_parse = None
    if args.parse_systems and not args.fused:
        ps = min(args.parse_systems, n_sys)
        off = torch.zeros(ps * NP + 1, dtype=torch.int64, device=dev)
        eng.generate_text_device(dname, seed, n_instr, first, ps, 0, off.data_ptr(), sp)
        torch.cuda.synchronize(dev)
        tbytes = int(off[-1].item())
        txt = torch.empty(tbytes + 64, dtype=torch.uint8, device=dev)
        eng.generate_text_device(dname, seed, n_instr, first, ps, txt.data_ptr(), off.data_ptr(), sp)
        ptr = torch.empty((ps, NP, n_instr), dtype=torch.int16, device=dev)
        pcn = torch.empty((ps, NP), dtype=torch.int32, device=dev)
        pst = torch.empty((ps, NP), dtype=torch.int32, device=dev)
        eng.parse_traces_device(txt.data_ptr(), off.data_ptr(), ps * NP, n_instr, ptr.data_ptr(),
                                pcn.data_ptr(), pst.data_ptr(), sp)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 3
        e0.record(stream)
        for _ in range(reps):
            eng.parse_traces_device(txt.data_ptr(), off.data_ptr(), ps * NP, n_instr,
                                    ptr.data_ptr(), pcn.data_ptr(), pst.data_ptr(), sp)
        e1.record(stream)
        torch.cuda.synchronize(dev)
        pms = e0.elapsed_time(e1) / reps
        ok = (int(pst.abs().sum().item()) == 0 and torch.equal(pcn, counts[:ps]) and
              torch.equal(ptr, traces[:ps]))
        pbytes = tbytes + ptr.numel() * 2 + pcn.numel() * 4 + off.numel() * 8
        trace_parse = dict(kernel="parse_kernel (core_n.txt text -> packed traces, fgets/sscanf semantics)",
                           systems=ps, text_bytes=tbytes, bytes=pbytes, ms=round(pms, 3),
                           per_unit="text bytes read + 2 B per packed instruction + 4 B count + 8 B offset per file written/read",
                           achieved_gbs=round(pbytes / pms / 1e6, 1), peak_gbs=HBM_PEAK_GBS,
                           frac=round(pbytes / pms / 1e6 / HBM_PEAK_GBS, 4),
                           parity="bit-exact vs gen_kernel traces" if ok else "MISMATCH")
        del txt, ptr, pcn, pst, off

    # printProcessorState of every node's final record, formatted on the GPU (fmt_kernel):
    # the dump/checksum writer phase, HBM-write-bound; timed separately, not part of `value`
    dump_stream = None
    if not args.no_dump:
        n_rec = n_sys * NP
        d_txt = torch.empty(n_rec * pydsm.DUMP_SLOT, dtype=torch.uint8, device=dev)
        d_len = torch.empty(n_rec, dtype=torch.int32, device=dev)
        eng.format_run_dumps_device(pydsm.VIEW_FINAL, 0, n_sys, d_txt.data_ptr(), d_len.data_ptr(), sp)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 3
        e0.record(stream)
        for _ in range(reps):
            eng.format_run_dumps_device(pydsm.VIEW_FINAL, 0, n_sys, d_txt.data_ptr(),
                                        d_len.data_ptr(), sp)
        e1.record(stream)
        torch.cuda.synchronize(dev)
        fms = e0.elapsed_time(e1) / reps
        fbytes = n_rec * (64 + pydsm.DUMP_SLOT + 4)
        text_bytes = int(d_len.sum().item())
        dump_stream = dict(kernel="fmt_kernel (printProcessorState text of every final node record)",
                           records=n_rec, text_bytes=text_bytes, bytes=fbytes, ms=round(fms, 3),
                           per_unit="64 B record read + %d B slot + 4 B length written per node" % pydsm.DUMP_SLOT,
                           achieved_gbs=round(fbytes / fms / 1e6, 1), peak_gbs=HBM_PEAK_GBS,
                           frac=round(fbytes / fms / 1e6 / HBM_PEAK_GBS, 4))
        del d_txt, d_len

    cdev = torch.device("cpu")                                  # gloo: host tensors

    def allreduce_counters(t):
        """A device dsm_counters vector summed over ranks (max for max_rounds), as a dict."""
        if group is not None:
            t = t.clone()
            group.allreduce_counters(t, sp)
            torch.cuda.synchronize(dev)
        else:
            t = reduce_counters(t.clone().to(cdev), dist if use_dist else None)
        return pydsm.counters_to_dict(t.cpu().numpy().view(np.uint64))

    if group is not None:
        el = torch.tensor([int(elapsed * 1e9)], dtype=torch.int64, device=dev)
        group.allreduce(el, 1, pydsm.RED_MAX, sp)
        torch.cuda.synchronize(dev)
        elapsed_max = int(el.item()) * 1e-9
    else:
        el = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
        if use_dist:
            dist.all_reduce(el, op=dist.ReduceOp.MAX)
        elapsed_max = float(el.item())
    local_c = pydsm.counters_to_dict(cnt.cpu().numpy().view(np.uint64))
    c = allreduce_counters(cnt)

    # handled messages per transactionType (assignment.c:20-34), parity only: the timed
    # kernels do not count types, so the same traces run once more, untimed, on a context
    # with DSM_F_TYPE_COUNTS (the one-pass lock-step kernel with per-type counters); its
    # totals must equal the timed run's messages and the reference's per-type totals
    type_pass = None
    if not args.fused and not args.no_types:
        teng = pydsm.Engine(NP, n_instr, ring_cap=args.ring, device=local, type_counts=True)
        tcnt = torch.zeros(pydsm.NCOUNTERS, dtype=torch.int64, device=dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        teng.run_packed_device(traces, counts, n_sys, None, tcnt, sp)
        e1.record(stream)
        torch.cuda.synchronize(dev)
        tli = teng.launch_info()
        teng.close()
        tc = allreduce_counters(tcnt)
        type_pass = dict(msgs_by_type=[tc[f"msgs_{t}"] for t in pydsm.TYPE_NAMES],
                         msgs=tc["msgs"], ms=round(e0.elapsed_time(e1), 3),
                         kernel=tli["kernels"] + " with DSM_F_TYPE_COUNTS (parity only, untimed)")

    # parity after the timed region, on every rank: the last step's per-system results of this
    # rank's shard against the reference's own handler text (its full-size aggregate:
    # counters, status counts, hash sums, position-sensitive result digest), then the job's
    # all-reduced aggregate against the reference's total over ids [0, world * n)
    res_host = out.cpu().numpy().view(pydsm.RESULT_DTYPE).reshape(-1)
    mine, verdict, shard_msg = shard_parity(dname, seed, n_instr, first, res_host, local_c)
    # the library's device fold of the same results (dsm_aggregate_device, what the C driver
    # all-reduces) must equal the host fold
    agg_dev = torch.zeros(pydsm.NAGG, dtype=torch.int64, device=dev)
    eng.aggregate_device(out, n_sys, first, agg_dev, sp)
    torch.cuda.synchronize(dev)
    dev_diff = pydsm.aggregate_diff(pydsm.agg_vec_to_dict(agg_dev.cpu().numpy().view(np.uint64)), mine)
    if dev_diff:
        verdict = "bad"
        shard_msg += "; DEVICE AGGREGATE MISMATCH: " + ",".join(dev_diff)
    print(f"bench.py rank {rank}: {shard_msg}", file=sys.stderr, flush=True)
    avec = torch.from_numpy(agg_to_vec(mine, verdict).view(np.int64).copy())
    if group is not None:       # dsm_aggregate layout: the shard tallies ride in its reserved slots
        avec = avec.to(dev)
        group.allreduce_aggregate(avec, sp)
        torch.cuda.synchronize(dev)
    else:
        avec = reduce_vector(avec.to(cdev), dist if use_dist else None, (AGG_MAX,))
    parity, parity_detail = job_parity(dname, seed, n_instr, world, n_sys,
                                       avec.cpu().numpy().view(np.uint64), c)
    if type_pass is not None:
        gold, _ = golden_for(dname, seed, n_instr, 0, world * n_sys)
        ok_sum = sum(type_pass["msgs_by_type"]) == c["msgs"] == type_pass["msgs"]
        if not ok_sum:
            parity += "; MSGS_BY_TYPE MISMATCH (sum != messages)"
        elif gold is not None and gold.get("msgs_by_type"):
            parity += ("; msgs_by_type == reference (13 types)"
                       if type_pass["msgs_by_type"] == gold["msgs_by_type"]
                       else "; MSGS_BY_TYPE MISMATCH vs reference")
        else:
            parity += "; msgs_by_type sums to messages (no reference per-type totals)"

    if rank == 0:
        K = args.steps
        value = c["msgs"] * K / elapsed_max
        kavg = float(np.mean(kms))
        alg_bytes = 2 * local_c["instrs"] + (32 + 4 * NP) * local_c["systems"]
        if args.fused:
            alg_bytes = 32 * local_c["systems"]
        ach = alg_bytes / (kavg * 1e-3) / 1e9
        li = eng.launch_info()
        # the packed path runs the transition kernel as two launches per step (budget pass +
        # resume pass, run_engine's two-pass schedule): bytes and time are per step, i.e. the
        # sum over both launches (rocprof lists 2 sim_kernel dispatches per step)
        launches = 2 if li.get("resume_form") else 1
        # which kernel of the fast-forward / plain pair ran (the trace scan's verdict, read
        # back by dsm_launch_info_get) and which resume pass followed the budget pass
        ff_picked = li.get("ff_picked") == 1 or args.fused
        serial = li.get("resume_form") == 2
        # the kernels that did the step's work, as the runtime launched them (the pair's picked
        # halves; dsm_launch_kernel_names), e.g. "budget=sim_kernel<8, 12, 4, false, 48, 5>
        # resume=ser_kernel<8, false>"
        roof = dict(bound="hbm", achieved=round(ach, 2), peak=HBM_PEAK_GBS, unit="GB/s",
                    frac=round(ach / HBM_PEAK_GBS, 6), traffic=None,
                    kernel=li["kernels"] + (" (fused generator" if args.fused else " (packed traces")
                    + (f"; budget pass {li['budget_rounds']} rounds" if launches == 2 else "")
                    + ("; resume in serial form, one lane per suspended system" if serial else
                       "; resume with the hit-run fast-forward" if ff_picked and launches == 2 else "")
                    + ")",
                    launches_per_step=launches,
                    algorithmic_bytes_per_launch=alg_bytes, kernel_ms_avg=round(kavg, 3),
                    per_unit="2 B per consumed packed instruction + 32 B result + 4*np B counts per system"
                             + ("; 'launch' = one step's budget + resume launches" if launches == 2 else ""))
        tr = traffic_from_profiles(args.config) or {}
        if serial and tr.get("sim_kernel") and tr.get("ser_kernel") and not args.fused:
            roof["traffic"] = int(tr["sim_kernel"]["bytes_per_launch"] + tr["ser_kernel"]["bytes_per_launch"])
            roof["traffic_source"] = tr["sim_kernel"].get("source") + " (budget pass sim_kernel + serial resume ser_kernel, one dispatch each per step)"
        elif tr.get("sim_kernel") and not args.fused and not serial:
            roof["traffic"] = int(tr["sim_kernel"].get("bytes_per_launch") * launches)
            roof["traffic_source"] = tr["sim_kernel"].get("source") + (
                " (per-dispatch average x 2 dispatches per step)" if launches == 2 else "")
        # the compute-side roof of the transition kernels that ran (VALU utilisation,
        # occupancy, waits, LDS bank conflicts beside the HBM fraction), from the PMC passes
        # under profiles/ (tools/issue.py -> profiles/pmc_issue.json): these kernels are bound
        # by a round's dependent instruction chain, not by HBM
        iss = issue_from_profiles(args.config) or {}
        ran = ["sim_kernel_budget"] + (["ser_kernel"] if serial else
                                       ["sim_kernel_ff"] if ff_picked and launches == 2 else [])
        if not args.fused and all(k in iss for k in ran):
            roof["issue"] = {k: iss[k] for k in ran}
            roof["issue_how"] = ("valu_busy = SQ_INSTS_VALU x 2 / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs); "
                                 "waves_per_simd = SQ_WAVE_CYCLES x 4 / (GRBM_GUI_ACTIVE / 8) / 1024; "
                                 "wait_frac / issue_stall_frac = SQ_WAIT_ANY / SQ_WAIT_INST_ANY over "
                                 "their sum with SQ_ACTIVE_INST_ANY; wait_per_wave_cycle = SQ_WAIT_ANY / "
                                 "SQ_WAVE_CYCLES; clock = GRBM_GUI_ACTIVE / 8 / wall")
        for phase, kname in ((trace_parse, "parse_kernel"), (dump_stream, "fmt_kernel"),
                             (trace_stream, "gen_kernel")):
            if phase is not None and tr.get(kname):
                phase["traffic"] = tr[kname].get("bytes_per_launch")
        # and system by system: the golden per-system prefix (tests/golden/ensemble/np8_<dist>.npy)
        gp = os.path.join(GOLDEN, "ensemble", f"np8_{dname}.npy")
        if first == 0 and os.path.exists(gp):
            g = np.load(gp)
            r = res_host[:len(g)]
            mine6 = np.stack([r["status"].astype(np.uint64), r["rounds"].astype(np.uint64),
                              r["msgs"].astype(np.uint64), r["instrs"].astype(np.uint64),
                              r["dump_hash"], r["final_hash"]], axis=1)
            parity += (f"; golden[0:{len(r)}] bit-exact" if np.array_equal(mine6, g[:len(r)])
                       else "; GOLDEN MISMATCH")
        cpu = cpu_port = None
        if world == 1 and not args.no_cpu:
            hc = host_cpu()
            threads = hc["threads"]
            cpu = cpu_baseline_reference(dname, n_instr, seed,
                                         min(args.cpu_ref_sample or n_sys, n_sys), threads)
            _, cpu_port = cpu_baseline(dname, n_instr, seed, min(args.cpu_sample or n_sys, n_sys),
                                       threads)
            if cpu is None:
                cpu, cpu_port = cpu_port, None
            for b in (cpu, cpu_port):
                if b is not None:
                    b["host"] = hc
            # the whole host: the systems are independent and the forked slices share nothing,
            # so the rate is linear in cores; checked by a second run of the reference leg on
            # half the processes over half the sample, then scaled to nproc (an estimate: the
            # pool gives this job a 16-CPU share, measured above)
            if cpu is not None and cpu["kind"] == "reference" and threads >= 2:
                half = cpu_baseline_reference(dname, n_instr, seed,
                                              max(1, min(args.cpu_ref_sample or n_sys, n_sys) // 2),
                                              threads // 2)
                if half is not None:
                    pc, pc_half = cpu["value"] / threads, half["value"] / (threads // 2)
                    cpu["per_core"] = round(pc, 1)
                    cpu["linearity"] = dict(cores=threads // 2, per_core=round(pc_half, 1),
                                            ratio=round(pc / pc_half, 4))
                    cpu["full_host_estimate"] = dict(
                        value=round(pc * hc["nproc"], 1), cores=hc["nproc"],
                        how=f"per-core rate at {threads} processes x nproc (estimate, not measured)")
        rec = {
            "metric": METRIC, "value": round(value, 1), "unit": UNIT, "n_gpus": world,
            "steps": K, "warmup": args.warmup, "ms_per_step": round(elapsed_max / K * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (counter-based generator, seed %d)" % seed,
            "config": {"workload": workload, "systems_per_gpu": n_sys, "np": NP,
                       "instr_per_node": n_instr, "dist": dname,
                       "parallelism": f"ensemble-dp{world}",
                       "traces": "fused generator (no HBM traces)" if args.fused else
                                 "packed u16 traces resident in HBM"},
            "roofline": roof,
            "cpu_baseline": cpu,
            "cpu_port": cpu_port,
            "trace_stream": trace_stream,
            "trace_parse": trace_parse,
            "dump_stream": dump_stream,
            "systems_per_s": round(c["systems"] * K / elapsed_max, 1),
            "instructions_per_s": round(c["instrs"] * K / elapsed_max, 1),
            "counters": {k: c[k] for k in ("msgs", "instrs", "rounds", "systems", "max_rounds",
                                           "overflow_reruns", "wave_rounds", "resumed",
                                           "ff_passes", "ff_steps", "ff_sample_instrs",
                                           "ff_sample_runs", "ser_macro_steps", "ser_iterations", "status_COMPLETED",
                                           "status_DEADLOCKED")},
            "msgs_by_type": dict(zip(pydsm.TYPE_NAMES, type_pass["msgs_by_type"])) if type_pass else None,
            "type_pass": {k: v for k, v in (type_pass or {}).items() if k != "msgs_by_type"} or None,
            "kernel_ms": [round(x, 3) for x in kms],
            "sum_final_hash": hex(c["sum_final_hash"]),
            "parity": parity,
            "parity_detail": parity_detail,
            "collective": (f"rccl ncclAllReduce issued by libdsm (dsm_group_*: counters, aggregate, "
                           f"elapsed max, barriers) over {world} rank(s)" if group is not None else
                           f"{backend} all_reduce of {pydsm.NCOUNTERS} counters over {world} rank(s)"
                           if use_dist else None),
            "launch": eng.launch_info(),
        }
        print(json.dumps(rec), flush=True)
    eng.close()
    if group is not None:
        group.close()
    if use_dist:
        dist.destroy_process_group()
    # a failed parity check fails the run: this rank's shard, and on rank 0 the job's line
    if verdict == "bad" or (rank == 0 and "MISMATCH" in parity):
        sys.exit(3)


if __name__ == "__main__":
    main()
