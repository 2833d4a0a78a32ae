/*
 * include/dsm.h -- C ABI of the MI355X-native ensemble coherence simulator (libdsm.so).
 *
 * The reference (ruubhagat/HP-Assignment-2, assignment.c) has no plugin or FFI API: its
 * whole boundary is the process contract `./cache_simulator <test_directory>` plus four
 * internal C functions.  Each entry point below names the reference interface it replaces:
 *
 *   dsm_parse_trace_file / dsm_load_test_dir  <- initializeProcessor   assignment.c:776-822
 *   dsm_parse_traces_device / dsm_parse_traces <- initializeProcessor's reader (:802-818) on
 *                                                the GPU, for whole ensembles of core files
 *   dsm_format_dump / dsm_write_dump          <- printProcessorState   assignment.c:824-876
 *   dsm_format_dumps_device / dsm_format_run_dumps_device / dsm_write_run_dumps
 *                                             <- printProcessorState, on the GPU, for whole
 *                                                ensembles (byte-identical text)
 *   dsm_run_* (lock-step ensemble engine)     <- the per-node loop of main (:135-699), the
 *                                                message switch (:177-566), instruction issue
 *                                                (:590-687), handleCacheReplacement
 *                                                (:742-773) and sendMessage (:711-739)
 *   dsm_get_node_state                        <- the processorNode snapshot handed to
 *                                                printProcessorState by value (:695)
 *
 * Conventions: plain C types only; every function returns 0 (DSM_OK) or a negative DSM_E_*
 * code (dsm_strerror); nothing throws across the ABI.  A dsm_ctx owns its device memory, is
 * bound to one GPU and must be used from one host thread at a time (not reentrant).  Its
 * device-side scratch (claim counters, suspended lists, the parser's EXACT-pass file list) is
 * shared by every call on it, so a ctx runs ONE asynchronous run or parse at a time, on one
 * stream: enqueue calls on the same ctx onto the same stream (stream order serialises them),
 * or use one ctx per concurrent stream.  The engine runs on hand-written gfx950 HIP kernels only: there is no CPU fallback, and when the
 * device cannot be used the run functions fail with DSM_E_DEVICE.
 */
#ifndef DSM_H
#define DSM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DSM_ABI_VERSION 5   /* 3: dsm_launch_info grew resume_form / budget_rounds / ff_picked;
                             4: dsm_counters grew to DSM_NCOUNTERS (ser_macro_steps), dsm_launch_info
                                names the kernels that ran (dsm_launch_kernel_names);
                             5: per-system aggregates (dsm_aggregate_*) and the multi-GPU group
                                over RCCL (dsm_group_*) */

#define DSM_MAX_NP 8             /* bitVector is one byte (README.md:51)                  */
#define DSM_CACHE_SIZE 4         /* CACHE_SIZE      assignment.c:10                        */
#define DSM_MEM_SIZE 16          /* MEM_SIZE        assignment.c:11                        */
#define DSM_REF_RING_CAP 256     /* MSG_BUFFER_SIZE assignment.c:12                        */
#define DSM_REF_MAX_INSTR 32     /* MAX_INSTR_NUM   assignment.c:13                        */
#define DSM_MAX_INSTR 4096       /* longest per-node trace the engine accepts               */
#define DSM_NTYPES 13            /* transactionType assignment.c:20-34                     */
#define DSM_MAX_ROUNDS (1u << 22)  /* active rounds before DSM_ROUND_LIMIT is reported */
#define DSM_DUMP_BASE 1954       /* printProcessorState text length with no EXCLUSIVE line    */
#define DSM_DUMP_MAX 1958        /* ... with four ("%8s" of "EXCLUSIVE" is 9 characters)       */
#define DSM_DUMP_SLOT 1968       /* bytes per record in GPU-formatted dump buffers (16 | slot) */

/* return codes */
enum {
    DSM_OK = 0,
    DSM_E_INVAL = -1,    /* bad argument or configuration                                  */
    DSM_E_DEVICE = -2,   /* no usable gfx950 device / HIP runtime error                     */
    DSM_E_NOMEM = -3,    /* device or host allocation failed                                */
    DSM_E_IO = -4,       /* trace or dump file could not be opened / written                */
    DSM_E_FORMAT = -5,   /* trace line the reference would not parse into an instruction    */
    DSM_E_STATE = -6,    /* e.g. dsm_get_node_state without DSM_F_SNAPSHOTS                  */
    DSM_E_RANGE = -7     /* address whose home node is >= np (assignment.c:90 would overrun) */
};

/* per-system status (dsm_sys_result.status bits 0..7); bits 8..15 = mask of dumped nodes */
enum {
    DSM_COMPLETED = 0,      /* every node issued all instructions and dumped (:688-697)     */
    DSM_DEADLOCKED = 1,     /* quiescent with some node still waitingForReply (:578-581)    */
    DSM_RING_OVERFLOW = 2,  /* an inbox would exceed MSG_BUFFER_SIZE (:715-724)              */
    DSM_ASSERT_FAILED = 3,  /* a reference assert() would have aborted (:189,:443,:489,...) */
    DSM_ROUND_LIMIT = 4     /* DSM_MAX_ROUNDS active rounds without quiescence             */
};

/* transactionType, assignment.c:20-34 (same numeric values) */
enum {
    DSM_READ_REQUEST = 0, DSM_WRITE_REQUEST, DSM_REPLY_RD, DSM_REPLY_WR, DSM_REPLY_ID, DSM_INV,
    DSM_UPGRADE, DSM_WRITEBACK_INV, DSM_WRITEBACK_INT, DSM_FLUSH, DSM_FLUSH_INVACK,
    DSM_EVICT_SHARED, DSM_EVICT_MODIFIED
};

/* synthetic address distributions (BASELINE.json configs) */
enum { DSM_DIST_UNIFORM = 0, DSM_DIST_HOT = 1, DSM_DIST_EVICT = 2 };

/* node-record views of a run (dsm_format_run_dumps_device) */
enum { DSM_VIEW_DUMP = 0,   /* snapshot when the node finished issuing (:695)              */
       DSM_VIEW_FINAL = 1   /* state when the system stopped                               */ };

/* config flags */
#define DSM_F_SNAPSHOTS 1u  /* keep per-node dump + final records of the last run          */
#define DSM_F_TIMING 2u     /* record HIP events around the transition kernel of each run     */
#define DSM_F_TYPE_COUNTS 4u /* count handled messages per transactionType (msgs_by_type)     */
#define DSM_F_ISSUE_TRACE 8u /* record every system's issue order (dsm_get_issue_trace)         */

/* act_thresh of dsm_set_schedule that means the plain lock-step schedule (the default) */
#define DSM_SCHED_LOCKSTEP 0x10000u

typedef struct dsm_config {
    int np;              /* NUM_PROCS: 4 or 8                                               */
    uint32_t max_instr;  /* per-node trace slot (stride) in instructions; multiple of 8,
                            <= DSM_MAX_INSTR                                                */
    uint32_t ring_cap;   /* inbox depth of the fast kernel: 0 (= 12), 4, 8, 12 or 16. Systems
                            that would overflow it are re-run on the device with the
                            reference depth 256; only overflow beyond 256 is reported.     */
    uint32_t flags;      /* DSM_F_*                                                         */
} dsm_config;

/* counter-based trace generator: instruction i of node n of system s depends only on
 * (seed, dist, np, s, n, i), so results do not depend on batching or GPU count. */
typedef struct dsm_gen {
    uint64_t seed;
    int dist;            /* DSM_DIST_*                                                      */
    uint32_t n_instr;    /* instructions per node, <= DSM_MAX_INSTR                         */
} dsm_gen;

/* per-system result, 32 bytes */
typedef struct dsm_sys_result {
    uint32_t status;     /* DSM_COMPLETED.. | dumped-node mask << 8                         */
    uint32_t rounds;     /* active lock-step rounds                                         */
    uint32_t msgs;       /* messages handled (transactions)                                 */
    uint32_t instrs;     /* instructions issued                                             */
    uint64_t dump_hash;  /* sum over dumped nodes of dsm_node_hash(node, dump, 15)          */
    uint64_t final_hash; /* sum over nodes of dsm_node_hash(node, final, 16)                */
} dsm_sys_result;

/* canonical node record, 64 bytes; field meanings from processorNode (assignment.c:70-81) */
typedef struct dsm_node_state {
    uint8_t memory[DSM_MEM_SIZE];      /* node.memory                                       */
    uint8_t dir_bv[DSM_MEM_SIZE];      /* directory[i].bitVector                            */
    uint8_t dir_state[DSM_MEM_SIZE];   /* directory[i].state: EM=0, S=1, U=2 (:18)          */
    uint8_t cache_addr[DSM_CACHE_SIZE];
    uint8_t cache_value[DSM_CACHE_SIZE];
    uint8_t cache_state[DSM_CACHE_SIZE]; /* MODIFIED=0, EXCLUSIVE=1, SHARED=2, INVALID=3    */
    uint8_t pending;                   /* pendingWriteValue                                 */
    uint8_t flags;                     /* bit0 waitingForReply, bit1 dumped                 */
    uint16_t issued;                   /* instructions issued (instructionIdx + 1)          */
} dsm_node_state;

/* aggregate counters (all sums except max_rounds); DSM_NCOUNTERS x uint64 */
#define DSM_NCOUNTERS 40
typedef struct dsm_counters {
    uint64_t msgs_by_type[DSM_NTYPES];   /* only with DSM_F_TYPE_COUNTS (else zero) */
    uint64_t msgs;
    uint64_t instrs;
    uint64_t rounds;
    uint64_t systems;
    uint64_t by_status[5];
    uint64_t sum_dump_hash;    /* mod 2^64 */
    uint64_t sum_final_hash;   /* mod 2^64 */
    uint64_t max_rounds;       /* max, not sum */
    uint64_t overflow_reruns;  /* systems re-run with the 256-deep inbox */
    uint64_t wave_rounds;      /* lock-step loop iterations summed over waves (cost model) */
    uint64_t resumed;          /* systems the two-pass schedule suspended and resumed      */
    uint64_t ff_passes;        /* hit-run fast-forward steps that advanced a system (the
                                * lock-step kernels' step (0); 0 when no fast-forward ran)  */
    uint64_t ff_steps;         /* fast-forward steps per wave (cost model)                  */
    uint64_t ff_sample_instrs; /* DSM_FF_AUTO: instructions of the sampled traces           */
    uint64_t ff_sample_runs;   /* ... of them ending a run of 8 hits (a private 4-line model) */
    uint64_t ser_macro_steps;  /* ABI 4: lone-node whole-transaction steps of the serial resume
                                * pass (dsm_serial.h ser_macro)                              */
    uint64_t ser_iterations;   /* ABI 5: wave iterations of the serial resume pass (cost model;
                                * wave_rounds holds them too, with the lock-step rounds)      */
    uint64_t reserved[6];      /* zero (probe builds: diagnostics)                            */
} dsm_counters;

typedef struct dsm_ctx dsm_ctx;

/* launch geometry of the last run (for measurement / roofline accounting) */
typedef struct dsm_launch_info {
    int grid_blocks;       /* persistent workgroups of the transition kernel               */
    int block_threads;
    int waves_per_cu;      /* resident waves per CU the occupancy query allowed            */
    int cus;
    int ring_cap;
    int lds_bytes_per_block;
    int resume_blocks;     /* two-pass schedule: workgroups of the resume pass that ran
                            * (0: none; the serial form runs one per CU, fewer when
                            * n_sys < 384 per CU, with a 384-KiB inbox spill area each)     */
    int budget_log2;       /* the plain budget pass's round budget, log2 (0: one pass)     */
    int late_log2;         /* the budget once a wave finds no new system, log2 (0: none)   */
    int round_limit_log2;  /* ROUND_LIMIT after 1 << this many active rounds               */
    int fmt_tile;          /* dump formatter tile (DSM_FMT at dsm_open)                   */
    int parse_bpl;         /* trace parser bytes per lane per window (DSM_PARSE_BPL)       */
    /* ABI 3: which passes ran.  With DSM_FF_AUTO the trace scan decides on the device, so
     * dsm_launch_info_get waits for the last run's stream to read its verdict. */
    int resume_form;       /* DSM_RESUME_*: the resume pass that ran                        */
    int budget_rounds;     /* the budget pass's effective budget in rounds (0: one pass):
                            * 1 << budget_log2, or the fast-forward budget (448) when the
                            * scan picked the hit-run fast-forward                           */
    int ff_picked;         /* 1 when the hit-run fast-forward kernel carried the run        */
    /* ABI 4: the kernels that did the work (the pair's picked halves), for measurement
     * labels: sim_kernel<np, ring_cap, block_threads / 64, gen, MODE, occ> */
    int np;
    int gen;               /* 1: the fused generator (dsm_run_generated*)                   */
    int occ;               /* the fast kernel's waves-per-EU bound (template OCC)            */
    int budget_mode;       /* MODE of the sim_kernel of the budget (or only) pass            */
    int resume_mode;       /* MODE of the lock-step resume sim_kernel; -1: ser_kernel or none */
    int ser_cap;           /* the serial resume ran ser_kernel<np, true> (inbox limit < 256) */
} dsm_launch_info;

enum { DSM_RESUME_NONE = 0, DSM_RESUME_LOCKSTEP = 1, DSM_RESUME_SERIAL = 2,
       DSM_RESUME_FASTFORWARD = 3 };

/* "budget=<kernel> resume=<kernel>" (or "run=<kernel>" for one pass) of a launch info, e.g.
 * "budget=sim_kernel<8, 12, 4, false, 48, 5> resume=ser_kernel<8, false>"; returns the
 * length, or DSM_E_INVAL if cap is too small (host only). */
int dsm_launch_kernel_names(const dsm_launch_info *info, char *buf, size_t cap);

/* ---- library ---------------------------------------------------------------------- */
int dsm_abi_version(void);
const char *dsm_strerror(int code);
int dsm_device_count(int *count);

/* ---- engine context (GPU) ---------------------------------------------------------- */
int dsm_open(int device, const dsm_config *cfg, dsm_ctx **out);
void dsm_close(dsm_ctx *ctx);
int dsm_launch_info_get(dsm_ctx *ctx, dsm_launch_info *info);

/* Host buffers: traces [n_sys][np][max_instr] packed u16 (bit15 WR, bits8-14 address,
 * bits0-7 value), counts [n_sys][np].  Copies in, runs, copies out, synchronises.
 * per_sys (n_sys entries) and out may be NULL; out is overwritten. */
int dsm_run_packed(dsm_ctx *ctx, const uint16_t *traces, const uint32_t *counts,
                   uint64_t n_sys, dsm_sys_result *per_sys, dsm_counters *out);

/* Device buffers (e.g. torch-owned HBM), asynchronous on `stream` (hipStream_t; NULL =
 * null stream).  d_results may be NULL; d_counters (device, one dsm_counters: DSM_NCOUNTERS
 * x uint64 = 320 bytes at ABI 4 -- a 32-slot buffer of ABI 3 is too small and would be written
 * past its end) is ACCUMULATED into.  No host synchronisation inside: every launch (including the two-pass
 * schedule's resume pass, which sizes itself on the device) is enqueued on `stream`.
 * Device traces are not validated: a count above max_instr is clamped to max_instr, and an
 * instruction whose home node (address >> 4) is >= np ends its system with
 * DSM_ASSERT_FAILED (the reference would index out of bounds, assignment.c:90). */
int dsm_run_packed_device(dsm_ctx *ctx, const uint16_t *d_traces, const uint32_t *d_counts,
                          uint64_t n_sys, dsm_sys_result *d_results,
                          dsm_counters *d_counters, void *stream);

/* GPU trace generator: writes d_traces [n_sys][np][max_instr] and d_counts [n_sys][np]
 * for systems first_sys .. first_sys+n_sys-1 (requires gen->n_instr <= max_instr). */
int dsm_generate_device(dsm_ctx *ctx, const dsm_gen *gen, uint64_t first_sys, uint64_t n_sys,
                        uint16_t *d_traces, uint32_t *d_counts, void *stream);

/* Engine with the generator fused in (instructions computed when issued; no trace bytes). */
int dsm_run_generated_device(dsm_ctx *ctx, const dsm_gen *gen, uint64_t first_sys,
                             uint64_t n_sys, dsm_sys_result *d_results,
                             dsm_counters *d_counters, void *stream);
int dsm_run_generated(dsm_ctx *ctx, const dsm_gen *gen, uint64_t first_sys, uint64_t n_sys,
                      dsm_sys_result *per_sys, dsm_counters *out);

/* Snapshot of node `node` of system `sys` of the last run (needs DSM_F_SNAPSHOTS):
 * `dump` = state when the node finished issuing (what printProcessorState prints, :695),
 * `final_state` = state when the system stopped.  Either pointer may be NULL. */
int dsm_get_node_state(dsm_ctx *ctx, uint64_t sys, int node, dsm_node_state *dump,
                       dsm_node_state *final_state);

/* Seeded schedule exploration for the following runs: in each round, a node that has an
 * action (Appendix A: inbox head, issue, dump) takes it only if the top 16 bits of
 * splitmix64(seed * 0x9E3779B97F4A7C15 + (sys << 26 ^ round << 3 ^ node)) are below
 * act_thresh, else it stalls that round -- another legal interleaving of the reference's
 * free-running OpenMP threads (:153-699).  A round counts while any node has an action.
 * act_thresh >= DSM_SCHED_LOCKSTEP restores the lock-step schedule.  sys is the system's
 * index in the run. */
int dsm_set_schedule(dsm_ctx *ctx, uint64_t seed, uint32_t act_thresh);

/* Issue order of system `sys` of the last run (needs DSM_F_ISSUE_TRACE): events in the
 * order the reference's DEBUG_INSTR printf (:595-598) would print them under the schedule
 * (round, then node): node << 16 | packed instruction.  *n = number of events (may exceed
 * cap; min(cap, *n) are copied). */
int dsm_get_issue_trace(dsm_ctx *ctx, uint64_t sys, uint32_t *events, uint32_t cap,
                        uint32_t *n);
/* DEBUG_INSTR lines ("Processor %d: instr type=%c, address=0x%02X, value=%d\n") of n
 * events; returns the length, or DSM_E_INVAL if cap is too small (host only). */
int dsm_format_issue_trace(const uint32_t *events, uint32_t n, char *buf, size_t cap);

/* Device time of the transition kernel of the last run (needs DSM_F_TIMING): HIP events
 * recorded on the run's own stream right before and after its launches.  The window holds
 * every launch of the budget and resume passes: with DSM_FF_AUTO on the packed path that is
 * the trace scan (ffscan_kernel, ~0.02 ms) and both kernels of each fast-forward / plain pair,
 * one of which exits at once (a few microseconds).  Waits for the stop event. */
int dsm_last_kernel_ms(dsm_ctx *ctx, float *ms);
/* The same for the last min(cap, runs, 64) runs, oldest first; *n = how many. */
int dsm_kernel_ms_history(dsm_ctx *ctx, float *ms, uint32_t cap, uint32_t *n);

/* Two-pass schedule of the packed path (bench mode): the budget pass suspends systems still
 * running after 1 << budget_log2 rounds (0 = one pass), 1 << late_log2 once a wave finds no
 * new system (0 = off), and -- where the serial pass resumes -- a system as soon as it is
 * quiet with one node left that can act (DSM_LONE / DSM_LONE_MIN at dsm_open); the resume
 * pass continues them -- in serial form, one system per lane (DSM_SERIAL=0 at dsm_open: the
 * lock-step resume), or, for traces the fast-forward verdict picks, the fast-forward
 * lock-step kernel (their budget pass: the plain kernel at the fast-forward budget).
 * Results never depend on it.  Defaults 12 / 0 (or DSM_BUDGET_LOG2 / DSM_LATE_LOG2 at
 * dsm_open); the fast-forward kernel's budget is 448 rounds (DSM_FF_BUDGET_ROUNDS, or
 * DSM_FF_BUDGET_LOG2 as a power of two; 0 = the plain budget). */
int dsm_set_budget(dsm_ctx *ctx, uint32_t budget_log2, uint32_t late_log2);
/* Round limit of the following runs: a system still active after 1 << limit_log2 rounds
 * stops with DSM_ROUND_LIMIT (1 <= limit_log2 <= 22; 0 = DSM_MAX_ROUNDS). */
int dsm_set_round_limit(dsm_ctx *ctx, uint32_t limit_log2);
/* Inbox limit of the following runs (MSG_BUFFER_SIZE, assignment.c:12; 1..256, 0 = 256): an
 * append beyond it ends the system with DSM_RING_OVERFLOW (the reference spins, :715-724). */
int dsm_set_inbox_limit(dsm_ctx *ctx, uint32_t cap);
/* Hit-run fast-forward of the following packed-path runs in the bench mode (no type counts,
 * issue trace or schedule exploration): DSM_FF_AUTO (default) samples the traces on the
 * device first and runs the fast-forward kernel only where nodes issue long runs of hits;
 * DSM_FF_ON / DSM_FF_OFF force it.  Results never depend on it (only time does); the
 * sample's counts are reported in dsm_counters.ff_sample_*. */
#define DSM_FF_OFF 0
#define DSM_FF_ON 1
#define DSM_FF_AUTO 2
int dsm_set_fast_forward(dsm_ctx *ctx, int mode);

/* ---- initializeProcessor's trace reader on the GPU (:802-818) ---------------------- *
 * n_files core files concatenated in d_text; file f is d_text[d_offsets[f] .. d_offsets[f+1])
 * (d_offsets has n_files + 1 entries) and is node f % np of system f / np.  Each file is
 * read as the reference reads it -- fgets(line, 20) chunks, each one instruction, scanned
 * with "RD %hhx" / "WR %hhx %hhu" -- into d_traces[f * max_instr ..] (packed u16),
 * d_counts[f] = instructions (at most cap <= max_instr) and d_status[f] (may be NULL) = 0 or
 * the error at the first failing chunk, which also ends the count there: DSM_E_FORMAT (not
 * RD/WR, or a conversion failed) or DSM_E_RANGE (home node >= np).  Asynchronous on `stream`;
 * it uses the ctx's device file list, so no other run or parse of the same ctx may be in
 * flight on another stream (see Conventions above). */
int dsm_parse_traces_device(dsm_ctx *ctx, const char *d_text, const uint64_t *d_offsets,
                            uint64_t n_files, uint32_t cap, uint16_t *d_traces,
                            uint32_t *d_counts, int32_t *d_status, void *stream);
/* the same from host buffers (offsets[f] index into text); traces [n_files][max_instr] */
int dsm_parse_traces(dsm_ctx *ctx, const char *text, const uint64_t *offsets, uint64_t n_files,
                     uint32_t cap, uint16_t *traces, uint32_t *counts, int32_t *status);
/* Synthetic core files in the shipped tests' format ("RD 0x%02x\n", "WR 0x%02x %u\n") for
 * the generator's instructions of systems first_sys .. first_sys+n_sys-1.  Always writes
 * d_offsets (n_sys*np + 1 entries; the last one is the total size); writes the text too
 * unless d_text is NULL (size query). */
int dsm_generate_text_device(dsm_ctx *ctx, const dsm_gen *gen, uint64_t first_sys, uint64_t n_sys,
                             char *d_text, uint64_t *d_offsets, void *stream);

/* ---- printProcessorState on the GPU (:824-876) ------------------------------------- *
 * Text of record k goes to d_text + k * DSM_DUMP_SLOT (16-byte aligned buffer), its length
 * (DSM_DUMP_BASE .. DSM_DUMP_MAX) to d_len[k]; the bytes after it in the slot are zero.  The
 * node id printed for record k is k % np.  Asynchronous on `stream`. */
int dsm_format_dumps_device(dsm_ctx *ctx, const dsm_node_state *d_states, uint32_t state_stride,
                            uint64_t n_states, char *d_text, uint32_t *d_len, void *stream);
/* the same for the np records of systems first_sys .. first_sys+n_sys-1 of the last run */
int dsm_format_run_dumps_device(dsm_ctx *ctx, int view, uint64_t first_sys, uint64_t n_sys,
                                char *d_text, uint32_t *d_len, void *stream);
/* GPU-format the dump records of system `sys` of the last run (needs DSM_F_SNAPSHOTS) and
 * write core_<n>_output.txt (:831) for every node n in node_mask into `dir` (NULL = CWD). */
int dsm_write_run_dumps(dsm_ctx *ctx, uint64_t sys, uint32_t node_mask, const char *dir);

/* ---- per-system aggregates (the shardable result of a run) ---------------------------- *
 * A run's per-system results folded into the reference's golden-aggregate view
 * (tests/golden/aggregates.json): sums over systems (mod 2^64), status counts, the max of
 * rounds, and a position-sensitive result digest -- the sum over systems of a fmix64 chain
 * over the system's ABSOLUTE id and its six result fields -- so the aggregates of the shards
 * of an ensemble (GPU g simulates ids [g*n, (g+1)*n)) merge into the job's by
 * addition, and a max for max_rounds.  DSM_NAGG x uint64, all-reducible as one vector. */
#define DSM_NAGG 16
#define DSM_AGG_MAX_SLOT 4       /* the one slot reduced by max (max_rounds)                  */
typedef struct dsm_aggregate {
    uint64_t systems;
    uint64_t msgs;             /* messages handled (transactions)                            */
    uint64_t instrs;
    uint64_t rounds;
    uint64_t max_rounds;       /* max, not sum                                               */
    uint64_t by_status[5];     /* DSM_COMPLETED .. DSM_ROUND_LIMIT                           */
    uint64_t sum_dump_hash;
    uint64_t sum_final_hash;
    uint64_t result_digest;
    uint64_t reserved[3];      /* zero (callers may carry their own sums here)               */
} dsm_aggregate;
/* d_results[0 .. n_sys) of the systems with ids first_sys, first_sys + 1, .. ACCUMULATED
 * into d_agg (device; zero it first for one run).  Asynchronous on `stream`. */
int dsm_aggregate_device(dsm_ctx *ctx, const dsm_sys_result *d_results, uint64_t n_sys,
                         uint64_t first_sys, dsm_aggregate *d_agg, void *stream);
/* the same on the host (no GPU needed); agg is overwritten */
int dsm_aggregate_results(const dsm_sys_result *res, uint64_t n_sys, uint64_t first_sys,
                          dsm_aggregate *agg);
/* one system's term of result_digest */
uint64_t dsm_result_digest(uint64_t sys_id, const dsm_sys_result *r);

/* ---- multi-GPU group: RCCL over xGMI --------------------------------------- *
 * Systems are independent, so an ensemble shards over GPUs with no data-path exchange; the
 * only collective is the final all-reduce of the counters and the aggregate (a few hundred
 * bytes).  A group is one RCCL communicator per GPU, created either
 *   - by one process per GPU: rank 0 calls dsm_group_unique_id and hands the id to every
 *     rank by any out-of-band channel, then each calls dsm_group_init_rank; or
 *   - by one process driving all GPUs (one host thread per device, as the reference runs
 *     one OpenMP thread per node): dsm_group_init_all, then each thread uses its own group.
 * The reductions run on the caller's stream (hipStream_t of the group's device), device
 * buffers in place, and return without a host wait.  Reference: there is no multi-GPU
 * equivalent in assignment.c; its only sharing is sendMessage's per-node queues (:711-739). */
#define DSM_GROUP_ID_BYTES 128
typedef struct dsm_group dsm_group;
enum { DSM_RED_SUM = 0, DSM_RED_MAX = 1 };
int dsm_group_unique_id(unsigned char id[DSM_GROUP_ID_BYTES]);
int dsm_group_init_rank(int device, int nranks, int rank, const unsigned char id[DSM_GROUP_ID_BYTES],
                        dsm_group **group);
int dsm_group_init_all(int ndev, const int *devices, dsm_group **groups /* [ndev] */);
int dsm_group_info(const dsm_group *group, int *rank, int *nranks, int *device);
int dsm_group_close(dsm_group *group);
/* n uint64 (mod 2^64 for DSM_RED_SUM) in place */
int dsm_group_allreduce(dsm_group *group, uint64_t *d_buf, size_t n, int op, void *stream);
/* dsm_counters in place: every slot summed except max_rounds (max) */
int dsm_group_allreduce_counters(dsm_group *group, dsm_counters *d_counters, void *stream);
/* dsm_aggregate in place: every slot summed except max_rounds (max) */
int dsm_group_allreduce_aggregate(dsm_group *group, dsm_aggregate *d_agg, void *stream);
/* returns once every rank's `stream` has reached this call (a one-element all-reduce, then
 * a wait for it on the host) */
int dsm_group_barrier(dsm_group *group, void *stream);

/* ---- boundary helpers (host only; no GPU needed) ----------------------------------- */
/* initializeProcessor's parser (:802-818): 20-byte fgets chunks, "RD %hhx" / "WR %hhx %hhu"
 * (mod-256 wrap), at most `cap` instructions (extra lines silently dropped as :805 does).
 * A chunk that is neither RD nor WR is DSM_E_FORMAT (the reference would count an
 * uninitialised instruction).  Missing file: DSM_E_IO. */
int dsm_parse_trace_file(const char *path, uint16_t *out, uint32_t cap, uint32_t *count);
/* tests/<dir_name>/core_<n>.txt for n < np, relative to the CWD (:794); addresses must
 * have home < np (DSM_E_RANGE).  traces [np][stride], counts [np]. */
int dsm_load_test_dir(const char *dir_name, int np, uint32_t cap, uint16_t *traces,
                      uint32_t stride, uint32_t *counts);
/* byte-exact printProcessorState text (:839-873); returns length, or DSM_E_INVAL if cap is
 * too small */
int dsm_format_dump(int node, const dsm_node_state *st, char *buf, size_t cap);
/* writes core_<node>_output.txt (:831) into directory `dir` (NULL = CWD) */
int dsm_write_dump(int node, const dsm_node_state *st, const char *dir);
/* 64-bit hash of the first nwords (15: dump view, 16: final view) u32 words of a record */
uint64_t dsm_node_hash(int node, const dsm_node_state *st, int nwords);

#ifdef __cplusplus
}
#endif
#endif
