/*
 * oracle/dsm_oracle.h -- TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline).
 * Clean-room C restatement of the reference protocol (ruubhagat/HP-Assignment-2,
 * assignment.c) under the deterministic lock-step schedule of SURVEY.md Appendix A.
 * Parity pinned by: the reference's own handler text driven under the same schedule
 * (oracle/_ref/ref_lockstep_np*, built by oracle/Makefile from /root/reference), the
 * lock-step dump md5s of SURVEY.md Appendix A, and the observed OpenMP outcome sets of the
 * unmodified reference binary (tests/golden/).
 */
#ifndef DSM_ORACLE_H
#define DSM_ORACLE_H
#include "dsm_common.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Simulate ONE system of np nodes.  trace[node*stride + i] packed u16 (dsm_common.h),
 * counts[node] instructions per node.  dump/fin (np records each) may be NULL.
 * by_type (13 counters) may be NULL and is accumulated into. */
int orc_run_system(int np, const uint16_t *trace, const uint32_t *counts, uint32_t stride,
                   uint32_t ring_cap, dsm_res *res, dsm_rec *dump, dsm_rec *fin,
                   uint64_t *by_type);

/* Batch over packed traces laid out [sys][node][stride]. */
int orc_run_packed(int np, const uint16_t *traces, const uint32_t *counts, uint32_t stride,
                   uint64_t n_sys, uint32_t ring_cap, dsm_res *res, dsm_rec *dump,
                   dsm_rec *fin, uint64_t *by_type, int nthreads);

/* Batch over generated traces (instructions produced lazily by dsm_gen_instr), systems
 * first_sys .. first_sys+n_sys-1.  OpenMP over systems when nthreads > 1. */
int orc_run_generated(int np, int dist, uint64_t seed, uint32_t n_instr, uint64_t first_sys,
                      uint64_t n_sys, uint32_t ring_cap, dsm_res *res, uint64_t *by_type,
                      int nthreads);

/* orc_run_packed plus seeded schedule exploration (dsm_sched_act with system id
 * first_sys + i; sched_thresh >= DSM_SCHED_LOCKSTEP = lock-step) and the issue order of every
 * system (issue [n_sys][issue_cap] of node << 16 | packed instruction, issue_n[n_sys]). */
int orc_run_packed_ex(int np, const uint16_t *traces, const uint32_t *counts, uint32_t stride,
                      uint64_t n_sys, uint32_t ring_cap, uint64_t sched_seed,
                      uint32_t sched_thresh, uint64_t first_sys, dsm_res *res, dsm_rec *dump,
                      dsm_rec *fin, uint32_t *issue, uint32_t issue_cap, uint32_t *issue_n,
                      int nthreads);

/* Round limit (active rounds before ST_ROUND_LIMIT) of the following runs; 0 = the default
 * DSM_ROUND_LIMIT.  Process-wide (test use). */
void orc_set_round_limit(uint32_t limit);

/* Fill traces [sys][node][n_instr] and counts [sys][node] from the generator. */
void orc_generate(int np, int dist, uint64_t seed, uint32_t n_instr, uint64_t first_sys,
                  uint64_t n_sys, uint16_t *traces, uint32_t *counts);

/* One action of one node (test hook for the per-transition model, tests/model/): a message
 * handled, or with type < 0 the instruction `ins` issued; *s updated, staged sends in out. */
int orc_step(int np, int me, dsm_rec *s, int type, uint16_t ins, int sender, int addr, int value,
             int bv, int r2, uint8_t (*out)[7], int *nout);

/* printProcessorState text (assignment.c:824-876) of one record; returns length or -1. */
int orc_format_dump(int node, const dsm_rec *r, char *buf, int cap);

uint64_t orc_hash_rec(int node, const dsm_rec *r, int nwords);

#ifdef __cplusplus
}
#endif
#endif
