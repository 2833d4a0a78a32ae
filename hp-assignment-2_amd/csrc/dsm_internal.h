/*
 * dsm_internal.h -- the engine context shared by the kernel translation units of libdsm.so
 * (dsm_engine.hip: transition engine; dsm_text.hip: trace parser and dump formatter).
 * Not part of the ABI.
 */
#ifndef DSM_INTERNAL_H
#define DSM_INTERNAL_H

#include <hip/hip_runtime.h>

#include "dsm.h"

struct SimArgs;   /* transition-kernel argument block (dsm_engine.hip) */

#define DSM_TIMING_RING 64

struct dsm_ctx {
    int device;
    dsm_config cfg;
    int ring;
    hipStream_t stream;
    int cus;
    unsigned int *d_ctrl;            /* claim shards (fast, fallback) + overflow count      */
    SimArgs *d_args;                 /* [0] fast kernel, [1] 256-deep re-run, [2] resume    */
    uint32_t *d_ovf_list;
    size_t ovf_cap;
    uint32_t *d_susp;                /* two-pass schedule: suspended node states             */
    size_t susp_cap;
    uint32_t *d_susp_list;           /*   and the suspended system ids                       */
    size_t susp_list_cap;
    uint32_t *d_spill;               /* serial resume: per-lane inbox spill FIFOs            */
    size_t spill_cap;
    uint16_t *d_traces;
    size_t traces_cap;
    uint32_t *d_counts;
    size_t counts_cap;
    dsm_sys_result *d_res;
    size_t res_cap;
    dsm_counters *d_cnt;
    uint2 *d_table;                  /* micro-op table, built on the host at open           */
    uint4 *d_recs;                   /* [sys][node][dump, final] node records of the last run */
    size_t recs_cap;
    uint64_t recs_n;
    /* DSM_F_TIMING: event pairs around the transition launches of the last DSM_TIMING_RING
     * runs (run k uses slot k % DSM_TIMING_RING) */
    hipEvent_t tev0[DSM_TIMING_RING], tev1[DSM_TIMING_RING];
    uint64_t runs_timed;
    dsm_launch_info info;
    /* the last run's pass choice when the device picks it (DSM_FF_AUTO): dsm_launch_info_get
     * reads the trace scan's verdict after waiting for last_st */
    hipStream_t last_st;
    int last_pair, last_use_ser, last_grid_fast, last_ser_blocks;
    uint32_t last_blog, last_thr_ff;
    /* two-pass schedule and round limit (dsm_set_budget / dsm_set_round_limit; defaults from
     * DSM_BUDGET_LOG2 / DSM_LATE_LOG2, read once at dsm_open) */
    uint32_t budget_log2, late_log2, round_limit_log2, inbox_limit;
    uint32_t ff_budget_log2;         /* the fast-forward kernel's budget (DSM_FF_BUDGET_LOG2) */
    uint32_t ff_budget_rounds;       /* ... as a round count, any value (DSM_FF_BUDGET_ROUNDS) */
    int ff_mode;                       /* DSM_FF_OFF / ON / AUTO */
    int serial;                        /* resume pass in serial form (ser_kernel; DSM_SERIAL) */
    uint32_t lone_rounds;              /* budget pass: suspend quiet-lone systems, checked every
                                        * this many rounds (DSM_LONE; 0: off)                  */
    uint32_t lone_min;                 /* ... not before this many rounds (DSM_LONE_MIN)        */
    /* dsm_text.hip tuning (DSM_FMT / DSM_PARSE_BPL, read once at dsm_open) */
    int fmt_tile, parse_bpl;
    uint64_t sched_seed;             /* dsm_set_schedule                                     */
    uint32_t sched_thresh;
    uint32_t *d_issue;               /* DSM_F_ISSUE_TRACE: [sys][np * max_instr] events      */
    size_t issue_cap_total;
    uint32_t *d_issue_n;
    size_t issue_n_cap;
    uint64_t issue_sys;
    /* dsm_text.hip */
    uint4 *d_dump_tpl;               /* np printProcessorState templates, DSM_DUMP_SLOT each  */
    char *d_text_tmp;                /* small staging for host-side dump writes              */
    uint32_t *d_len_tmp;
    char *d_parse_buf;               /* dsm_parse_traces (host text) staging                 */
    size_t parse_cap;
    uint64_t *d_parse_off;
    size_t parse_off_cap;
    uint32_t *d_parse_list;          /* parse_kernel: [0] files for the EXACT pass, then ids  */
    size_t parse_list_cap;
};

#define HIPCK(x) do { if ((x) != hipSuccess) return DSM_E_DEVICE; } while (0)

/* dsm_text.hip: called by dsm_close */
void dsm_text_release(dsm_ctx *c);

template <typename T>
static inline int dsm_ensure(T **p, size_t *cap, size_t need) {
    if (*cap >= need && *p) return DSM_OK;
    if (*p) { (void)hipFree(*p); *p = nullptr; *cap = 0; }
    if (hipMalloc((void **)p, need * sizeof(T)) != hipSuccess) { *p = nullptr; return DSM_E_NOMEM; }
    *cap = need;
    return DSM_OK;
}

#endif
