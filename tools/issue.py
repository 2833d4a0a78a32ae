#!/usr/bin/env python3
"""tools/issue.py <prof_dir> <config> -- the compute-side roof of the transition kernels from the
rocprofv3 SQ / wait passes written by tools/profile.sh, folded into profiles/pmc_issue.json
under <config> for bench.py's roofline "issue" field (VALU utilisation, LDS bank
conflicts and occupancy beside the HBM fraction).

Per dispatch of each transition kernel (the immediate-exit half of a fast-forward / plain pair
is dropped: dispatches under 1 ms), from the pmc_sq pass (one dispatch's counters share its
Start/End timestamps):
  clock_ghz        = GRBM_GUI_ACTIVE / 8 XCDs / wall              (MI355X_MICROARCH.md, DVFS)
  valu_busy        = SQ_INSTS_VALU x 2 cycles / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)
                     (a wave64 VALU instruction holds a SIMD's issue 2 cycles at full rate)
  waves_per_simd   = SQ_WAVE_CYCLES x 4 / (GRBM_GUI_ACTIVE / 8) / 1024
                     (SQ_WAVE_CYCLES counts quad-cycles: the mean resident waves per SIMD)
and from the pmc_wait pass (SQ_WAIT_ANY + SQ_WAIT_INST_ANY + SQ_ACTIVE_INST_ANY ~ the
wave-cycles):
  wait_frac        = SQ_WAIT_ANY / that sum        (waves parked on a counter: s_waitcnt)
  wait_per_wave_cycle = SQ_WAIT_ANY / SQ_WAVE_CYCLES (the SQ pass's per-dispatch mean)
  issue_stall_frac = SQ_WAIT_INST_ANY / that sum   (waves ready but not issued)
  lds_conflict_per_lds_inst = SQ_LDS_BANK_CONFLICT / SQ_ACTIVE_INST_LDS
Averages over the dispatches; the per-launch instruction counts ride along."""
import collections
import csv
import glob
import json
import os
import sys

SIMDS, XCDS = 1024, 8
# the plain budget kernel: M_NOFF (16) when the fast-forward kernel resumes, M_NOFF | M_SERB (48)
# when the serial pass does
KERNELS = {"sim_kernel_budget": ("::sim_kernel<8, 12, 4, false, 16, 5>", "::sim_kernel<8, 12, 4, false, 48, 5>"),
           "sim_kernel_ff": ("::sim_kernel<8, 12, 4, false, 0, 5>",),
           "ser_kernel": ("::ser_kernel<8, false>",)}


def dispatches(path, pattern):
    """{dispatch id: (wall ns, {counter: value})} of the kernels matching one of the patterns."""
    out = {}
    for f in glob.glob(os.path.join(path, "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if not any(p in r["Kernel_Name"] for p in pattern):
                continue
            d = out.setdefault(r["Dispatch_Id"], [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]),
                                                  collections.defaultdict(float)])
            d[1][r["Counter_Name"]] += float(r["Counter_Value"])
    return {k: v for k, v in out.items() if v[0] >= 1_000_000}


def summarize(d, pattern):
    sq, wt = dispatches(os.path.join(d, "pmc_sq"), pattern), dispatches(os.path.join(d, "pmc_wait"), pattern)
    if not sq:
        return None
    rows = []
    for wall, c in sq.values():
        cyc = c["GRBM_GUI_ACTIVE"] / XCDS
        rows.append(dict(ms=wall / 1e6, clock_ghz=cyc / wall, valu_busy=c["SQ_INSTS_VALU"] * 2 / (cyc * SIMDS),
                         waves_per_simd=c["SQ_WAVE_CYCLES"] * 4 / cyc / SIMDS, waves=c["SQ_WAVES"],
                         valu=c["SQ_INSTS_VALU"], salu=c["SQ_INSTS_SALU"], lds=c["SQ_INSTS_LDS"],
                         wave_cycles=c["SQ_WAVE_CYCLES"]))
    wrows = []
    wave_cycles = sum(r["wave_cycles"] for r in rows) / len(rows)
    for _, c in wt.values():
        tot = c["SQ_WAIT_ANY"] + c["SQ_WAIT_INST_ANY"] + c["SQ_ACTIVE_INST_ANY"]
        wrows.append(dict(wait_frac=c["SQ_WAIT_ANY"] / tot, issue_stall_frac=c["SQ_WAIT_INST_ANY"] / tot,
                          # the verdict's form: SQ_WAIT_ANY / SQ_WAVE_CYCLES (both quad-cycles; the
                          # two counters come from separate passes: the SQ pass's per-dispatch mean)
                          wait_per_wave_cycle=c["SQ_WAIT_ANY"] / max(wave_cycles, 1.0),
                          lds_bank_conflict_cycles=c["SQ_LDS_BANK_CONFLICT"],
                          lds_conflict_per_lds_inst=c["SQ_LDS_BANK_CONFLICT"] / max(c["SQ_ACTIVE_INST_LDS"], 1.0)))
    avg = lambda rs, k: sum(r[k] for r in rs) / len(rs)
    out = {k: avg(rows, k) for k in rows[0]}
    if wrows:
        out.update({k: avg(wrows, k) for k in wrows[0]})
    rnd = {"ms": 3, "clock_ghz": 3, "valu_busy": 4, "waves_per_simd": 3, "wait_frac": 4, "wait_per_wave_cycle": 4,
           "issue_stall_frac": 4, "lds_conflict_per_lds_inst": 4}
    out = {k: (round(v, rnd[k]) if k in rnd else int(v)) for k, v in out.items()}
    out["dispatches"] = len(rows)
    out["source"] = f"{d}/pmc_sq + pmc_wait (rocprofv3, separate passes)"
    return out


def main():
    d, config = sys.argv[1], sys.argv[2]
    res = {k: s for k, pat in KERNELS.items() if (s := summarize(d, pat))}
    p = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles", "pmc_issue.json")
    try:
        allv = json.load(open(p))
    except (OSError, ValueError):
        allv = {}
    allv[config] = res
    json.dump(allv, open(p, "w"), indent=1, sort_keys=True)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
