/*
 * dsm_engine.hip -- gfx950 (MI355X / CDNA4) kernels + C-ABI runtime of the ensemble
 * coherence simulator (libdsm.so).  See DESIGN.md for the layout and rooflines.
 *
 * What is simulated: the DASH-like directory MESI protocol of ruubhagat/HP-Assignment-2
 * (assignment.c): the per-node loop of main (:153-699) = inbox drain + 13-way message switch
 * (:177-566) + one-instruction issue (:590-687) + dump-once (:688-697),
 * handleCacheReplacement (:742-773) and sendMessage (:711-739), run under the deterministic
 * lock-step schedule on an ensemble of independent systems.
 *
 * Mapping (one wave64 = 64/NP systems, one lane = one node):
 *   - per-node registers: directory states (2 bits x 16), cache addresses / values (one byte
 *     per line), cache states (2 bits x 4), control word, counters;
 *   - per-node LDS column s_mb[wave][block/2][lane] (one dword per lane holds two blocks'
 *     memory byte | bitVector byte << 8), so a message touches its home block with one
 *     ds_read_u16 / ds_write_b16 (bank = lane % 32: conflict-free) instead of a runtime
 *     byte select over 8 registers;
 *   - inboxes: LDS rings s_ring[wave][slot][lane] (bank = lane % 32, conflict-free);
 *   - a round: every lane takes one action (predicated data flow, no per-type branches),
 *     writes <= 2 outgoing words to LDS and ORs their bits into the receivers' receive masks
 *     (LDS atomics); each receiver appends the words addressed to it in ascending
 *     (sender, word) order -- the reference's (sender, program order) delivery;
 *   - per-system termination by wave ballot; finished systems are replaced from sharded
 *     device work counters (persistent kernel), so lanes never idle on a long-tail system;
 *   - traces are read as 16-byte chunks per lane (current + prefetched next) from HBM;
 *   - systems whose inbox would exceed the fast ring are re-run by the same kernel built
 *     with the reference's 256-deep inbox, so results never depend on the fast ring size.
 */
#include <hip/hip_runtime.h>

#include <type_traits>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "dsm.h"
#ifndef SIM_BF
#define SIM_BF 0            /* A/B: bit 0 the first receive-mask ORs without a branch, bit 1 the
                               first destination index as a mask select (dsm_table.h) */
#endif
#include "dsm_table.h"
#include "dsm_internal.h"
#include "dsm_gen.h"
#include "dsm_serial.h"

/* Kernel arguments live in device memory (not the kernarg segment): the hot loop needs
 * almost none of them, and loads from a plain global pointer are not hoisted into SGPRs
 * that would then stay live across the whole loop. */
struct SimArgs {
    const uint16_t *traces;     /* [sys][np][stride] packed u16 (not GEN)                 */
    const uint32_t *counts;     /* [sys][np] (not GEN)                                     */
    uint32_t stride;
    uint32_t n_instr;           /* GEN: instructions per node                              */
    uint64_t n_sys;             /* systems (when d_n == nullptr)                           */
    const unsigned int *d_n;    /* list mode: device-resident count                        */
    const uint32_t *list;       /* list mode: system indices                               */
    uint64_t first_sys;         /* GEN: global id of system index 0                        */
    uint64_t seed;
    int dist;
    dsm_sys_result *results;    /* the transition kernel writes the first 16 bytes        */
    uint4 *recs;                /* [sys][node][2] x 64 B: dump record, final record       */
    unsigned long long *counters;   /* dsm_counters (device), accumulated into by atomics at
                                     * workgroup exit (integer sums: order-independent)   */
    unsigned int *claim;            /* 8 shard counters, 32 words apart                     */
    uint32_t *ovf_list;             /* fast kernel: systems handed to the 256-deep re-run   */
    unsigned int *ovf_count;
    const uint2 *table;             /* micro-op table (dsm_table.h), DT_TABLE_WORDS words   */
    uint64_t sched_seed;            /* M_SX: seeded schedule exploration (dsm_set_schedule)  */
    uint32_t sched_thresh;
    uint32_t issue_cap;             /* M_TR: events per system                               */
    uint32_t *issue;                /* M_TR: [sys][issue_cap] node << 16 | packed instruction */
    uint32_t *issue_n;              /* M_TR: [sys] events                                    */
    /* two-pass schedule (run_engine): a budget pass suspends every system still running
     * after 1 << rsh rounds, a resume pass continues them from their saved state */
    uint32_t rsh;                   /* round-limit test: rounds >> rsh != 0                  */
    uint32_t budget;                /* budget pass: suspend at 1 << rsh rounds               */
    uint32_t resume;                /* resume pass: start() restores a suspended system      */
    uint32_t ffsel;                 /* one of a fast-forward / plain pair of launches: run only
                                     * if scan's verdict picks this kernel (ffscan_kernel)    */
    const uint32_t *scan;           /* [sampled instructions, 8-hit-run ends] (ffscan_kernel) */
    uint32_t late_rsh;              /* budget pass: the budget once a wave finds no new work  */
    uint32_t *susp;                 /* [sys][word][node] suspended state (susp_words)        */
    uint32_t *susp_list;            /* budget pass: suspended system ids                     */
    unsigned int *susp_count;
    unsigned int *susp_long;        /* serial-form budget pass: systems of the long class, listed
                                     * from the list's top down (SER_LONG); the serial pass
                                     * claims them first                                     */
    uint32_t susp_cap;              /* the list's capacity (systems in the run)              */
    uint32_t lim_rsh;               /* round limit = 1 << lim_rsh (DSM_MAX_ROUNDS, or
                                     * dsm_set_round_limit): ROUND_LIMIT at that many rounds */
    uint32_t icap;                  /* inbox limit (MSG_BUFFER_SIZE = 256, or
                                     * dsm_set_inbox_limit): RING_OVERFLOW beyond it        */
    uint32_t susp_ring;             /* resume pass: ring depth of the suspended states       */
    uint32_t *spill;                /* serial resume: [lane][S_SPILL] queue spill FIFOs      */
    uint32_t thr_ff;                /* budget pass, fast-forward kernel: suspend at this many
                                     * rounds (0: at 1 << rsh)                               */
    uint32_t lone;                  /* budget pass with a serial resume: every `lone` rounds,
                                     * suspend the systems that have become quiet-lone (one
                                     * node may act, nothing queued) -- the serial pass's
                                     * macro-step takes them (0: off)                        */
    uint32_t lone_min;              /* ... once they have run at least this many rounds        */
    uint32_t serfmt;                /* budget pass: suspended states in serial form (ssusp_words)
                                     * unless the fast-forward pair's pick resumes them      */
    uint32_t split;                 /* budget pass of the pair with a serial resume: the M_SERB
                                     * plain kernel and the one without are both launched    */
};
/* the argument blocks of one run, written to device memory by args_kernel (stream-ordered:
 * no pinned staging whose reuse would need a host wait) */
struct SimArgsPack { SimArgs a[3]; };


#define DEVI __device__ __forceinline__

/* s_waitcnt vmcnt(0) with expcnt / lgkmcnt left open, as the raw immediate of the gfx9 encoding
 * (vmcnt bits 3:0 and 15:14, expcnt 6:4, lgkmcnt 11:8): it means something else on gfx10+,
 * and this library is built for gfx950 only */
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "dsm_engine.hip targets gfx950 (raw gfx9 s_waitcnt encodings)"
#endif
DEVI void wait_vmcnt0() { __builtin_amdgcn_s_waitcnt(0x0F70); }
/* a wave-uniform value stated as such (v_readfirstlane): branches on it compile to scalar
 * branches, not exec-masked regions, whatever the compiler's uniformity analysis concluded */
DEVI uint32_t uni32(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
DEVI uint64_t uni64(uint64_t x) { return ((uint64_t)uni32((uint32_t)(x >> 32)) << 32) | uni32((uint32_t)x); }

#ifndef TRAFFIC_PROBE
#define TRAFFIC_PROBE 0     /* traffic attribution builds (results invalid): 1 no serial pass, 2 and
                               no serial-form suspend records (tools/traffic_streams.sh) */
#endif
#ifndef SIM_UNI
#define SIM_UNI 1           /* the suspend-on-lone budget pass's per-round end test as one per-lane
                               ballot, not 64-bit mask arithmetic (0: the mask form everywhere) */
#endif
#ifndef SIM_RFL
#define SIM_RFL 1           /* the round loop's wave-uniform values (the live mask, the end test,
                               the lone-check countdown) pinned uniform with readfirstlane */
#endif
#ifndef SIM_R2
#define SIM_R2 0            /* plain budget kernels: a third trace chunk in registers and the refill
                               as one 32-B load every 16 instructions (half the chunk loads, each
                               a line fetch: the scattered 16-B loads find no line in L2) */
#endif
#ifndef REC_PROBE
#define REC_PROBE 0         /* probe build (hashes invalid): no node records and no digest pass, to
                               time what the records cost the step */
#endif
#ifndef SER_LONG
#define SER_LONG 0          /* the serial pass claims lone systems with this many instructions left
                               (and multi-node ones) first, the rest last-suspended first (0: all
                               last-suspended first) */
#endif
#ifndef SIM_TAILPROBE
#define SIM_TAILPROBE 0     /* budget-pass wave end-time histogram (probe build, results exact;
                               tools/tail_probe.py) */
#endif
#ifndef FF_LONG
#define FF_LONG 1           /* fast-forward runs past the 8-instruction window */
#endif
#ifndef FF_LONG_U
#define FF_LONG_U 8         /* trace chunks per step of that scan (hot, C4: 1 / 2 / 4 / 6 / 8 -> 49.6 / 39.3 / 34.1 / 32.6 / 32.1 ms) */
#endif

namespace {

using namespace dsmg;

/* transactionType (assignment.c:20-34) plus the local actions of one round */
enum : uint32_t {
    T_RREQ = 0, T_WREQ = 1, T_RRD = 2, T_RWR = 3, T_RID = 4, T_INV = 5, T_UPG = 6,
    T_WBINV = 7, T_WBINT = 8, T_FLUSH = 9, T_FLINV = 10, T_EVS = 11, T_EVM = 12,
    OP_RD = 13, OP_WR = 14, OP_DUMP = 15, OP_IDLE = 16
};

/* ctl word: bits 0-7 pendingWriteValue, then flags */
constexpr uint32_t C_WAIT = DT_CTL_WAIT, C_DUMPED = 1u << 9, C_OVF = 1u << 10, C_ASSERT = DT_CTL_ASSERT;

/* counter slots (dsm_counters order) */
enum { K_MSGS = 13, K_INSTRS = 14, K_ROUNDS = 15, K_SYSTEMS = 16, K_STATUS = 17, K_DHASH = 22,
       K_FHASH = 23, K_MAXR = 24, K_OVFRERUN = 25, K_WROUNDS = 26, K_RESUMED = 27,
       K_FFPASS = 28, K_FFITER = 29, K_SCANI = 30, K_SCANR = 31, K_N = 32,
       K_SERMAC = 32 /* ser_kernel only, added straight to the device counters */,
       K_SERIT = 33  /* ser_kernel only: its wave iterations (dsm_counters.ser_iterations)  */,
       K_SERPROBE = 34 /* SIM_TAILPROBE builds: the serial pass's wave end-time histogram, 34-39 */ };
static_assert(sizeof(dsm_counters) == DSM_NCOUNTERS * 8 && K_SERMAC < DSM_NCOUNTERS, "dsm_counters slots");
constexpr uint32_t RSH_MAX = 22;    /* 1 << 22 == DSM_MAX_ROUNDS */
static_assert((1u << RSH_MAX) == DSM_MAX_ROUNDS, "DSM_MAX_ROUNDS");
/* suspended node state: memory/bitVector (8), lines (4), ring (RING), dst, ctl, ip, nins, rh,
 * nmsg, rounds (7), trace chunks cur, nxt (8) */
constexpr int susp_words(int ring) { return 27 + ring; }
/* the suspended state in serial form (a budget pass whose resume pass is ser_kernel): one
 * contiguous record per system, so the resume reads it with 16-byte row loads --
 *   [0, 96)    the serial pass's LDS column (dsm_serial.h S_MB .. S_CT), as it will be;
 *   [96, 104)  per node: ring head | count << 8;  [104, 112) instructions in the trace;
 *   [112, 120) messages received;  [120] rounds;
 *   [121]      a lone system: its node | 0x100 (else 0), and [124, 128) / [128, 132) that
 *              node's trace chunk ip >> 3 and the next (the lock-step shift register cur,
 *              instructions ip.. in its low half-words, and nxt), so the serial pass's first
 *              macro-step has its instruction at hand;
 *   [136, 136 + 8 RING)  per node: its queued ring entries, oldest first (count of them). */
constexpr int SSUSP_HDR = 136;
constexpr int ssusp_words(int ring) { return SSUSP_HDR + 8 * ring; }

constexpr uint64_t NO_SYS = ~0ull;
constexpr uint32_t DSM_LINE_INIT = 0xFFu | (3u << 16);   /* address 0xFF, value 0, INVALID */
constexpr int FB_RING = 256;        /* MSG_BUFFER_SIZE, assignment.c:12 */

/* ---- small bit-field helpers ------------------------------------------------------- */
DEVI uint32_t get2(uint32_t w, uint32_t i) { return __builtin_amdgcn_ubfe(w, i * 2, 2); }
DEVI uint32_t set2(uint32_t w, uint32_t i, uint32_t v) {
    const uint32_t sh = i * 2;
    return (w & ~(3u << sh)) | (v << sh);
}

/* message words: dsm_table.h (dt_issue_word, dt_decode, dt_ring_entry) */

/* ---- hashing / generator (definitions in DESIGN.md; pinned by tests) ----------------- */
DEVI uint64_t fmix64(uint64_t z) {
    z ^= z >> 33; z *= 0xff51afd7ed558ccdULL;
    z ^= z >> 33; z *= 0xc4ceb9fe1a85ec53ULL;
    z ^= z >> 33;
    return z;
}
struct Node {
    uint32_t dst;     /* directory states, 2 bits per block                                 */
    uint32_t ctl;     /* pending | C_* flags                                                */
    uint32_t ip;      /* instructions issued                                                */
    uint32_t nins;    /* instructions in this node's trace                                  */
    uint32_t rh;      /* inbox head (bits 0-7) | count << 8                                 */
    uint32_t nmsg;    /* messages handled                                                   */
};

/* global-address-space views: a generic (flat) access is counted in both vmcnt and lgkmcnt
 * and completes out of order, so every later wait on memory, or on any LDS access, becomes
 * vmcnt(0) lgkmcnt(0) while one is in flight */
typedef uint32_t v4u32 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) uint32_t GU32;    /* global (not flat) accesses */
typedef __attribute__((address_space(1))) v4u32 GV4;
/* canonical 64-byte record (dsm_node_state) word i; mem / bv words come from LDS */
DEVI uint32_t rec_word(const Node &nd, const uint32_t (&mb)[8], const uint32_t (&ln)[4], uint32_t flags, int i) {
    switch (i) {
    case 0: case 1: case 2: case 3: case 4: case 5: case 6: case 7: return mb[i];
    case 8: case 9: case 10: case 11: {
        const uint32_t e = nd.dst >> (8 * (i - 8));
        return (e & 3u) | (((e >> 2) & 3u) << 8) | (((e >> 4) & 3u) << 16) | (((e >> 6) & 3u) << 24);
    }
    case 12: return __builtin_amdgcn_perm(__builtin_amdgcn_perm(ln[3], ln[2], 0x0C0C0400u),
                                          __builtin_amdgcn_perm(ln[1], ln[0], 0x0C0C0400u), 0x05040100u);
    case 13: return __builtin_amdgcn_perm(__builtin_amdgcn_perm(ln[3], ln[2], 0x0C0C0501u),
                                          __builtin_amdgcn_perm(ln[1], ln[0], 0x0C0C0501u), 0x05040100u);
    case 14:
        return __builtin_amdgcn_perm(__builtin_amdgcn_perm(ln[3], ln[2], 0x0C0C0602u),
                                     __builtin_amdgcn_perm(ln[1], ln[0], 0x0C0C0602u), 0x05040100u);
    default: return (nd.ctl & 0xFFu) | (flags << 8) | (nd.ip << 16);
    }
}
/* memory (words 0-3) and bitVector (words 4-7) bytes of this lane's node, from LDS */
template <int WAVES>
DEVI void load_mb(const uint32_t (&smb)[WAVES][8][64], uint32_t wv, uint32_t lane,
                  uint32_t (&mb)[8]) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t x = smb[wv][2 * k][lane], y = smb[wv][2 * k + 1][lane];
        /* x = b0 | v0 << 8 | b1 << 16 | v1 << 24, y likewise for blocks 4k+2, 4k+3 */
        mb[k] = __builtin_amdgcn_perm(y, x, 0x06040200u);      /* bytes b0 b1 b2 b3 */
        mb[4 + k] = __builtin_amdgcn_perm(y, x, 0x07050301u);  /* bytes v0 v1 v2 v3 */
    }
}
/* store this lane's 64-byte node record (dsm_node_state) */
template <int WAVES>
DEVI void store_rec(uint4 *dst, const Node &nd, const uint32_t (&smb)[WAVES][8][64],
                    const uint32_t (&sln)[WAVES][4][64], uint32_t wv, uint32_t lane, uint32_t flags) {
    const uint32_t ln[4] = {sln[wv][0][lane], sln[wv][1][lane], sln[wv][2][lane], sln[wv][3][lane]};
    uint32_t mb[8];
    load_mb<WAVES>(smb, wv, lane, mb);
    dst[0] = make_uint4(mb[0], mb[1], mb[2], mb[3]);
    dst[1] = make_uint4(mb[4], mb[5], mb[6], mb[7]);
    dst[2] = make_uint4(rec_word(nd, mb, ln, flags, 8), rec_word(nd, mb, ln, flags, 9),
                        rec_word(nd, mb, ln, flags, 10), rec_word(nd, mb, ln, flags, 11));
    dst[3] = make_uint4(rec_word(nd, mb, ln, flags, 12), rec_word(nd, mb, ln, flags, 13),
                        rec_word(nd, mb, ln, flags, 14), rec_word(nd, mb, ln, flags, 15));
}

template <int NP>
DEVI uint32_t gsum32(uint32_t x) {
#pragma unroll
    for (int o = 1; o < NP; o <<= 1) x += __shfl_xor(x, o, 64);
    return x;
}
template <int NP>
DEVI uint64_t gsum64(uint64_t x) {
#pragma unroll
    for (int o = 1; o < NP; o <<= 1) {
        const uint32_t lo = __shfl_xor((uint32_t)x, o, 64), hi = __shfl_xor((uint32_t)(x >> 32), o, 64);
        x += ((uint64_t)hi << 32) | lo;
    }
    return x;
}
/* 16-byte trace chunk load through the global address space: a generic (flat) load is
 * counted in both vmcnt and lgkmcnt and completes out of order, so every later wait on it,
 * or on any LDS access, becomes vmcnt(0) lgkmcnt(0). */
DEVI uint32_t gatomic_add(GU32 *p, uint32_t v) {
    return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
DEVI uint4 ld16(const uint16_t *p) {
    const v4u32 v = *(const __attribute__((address_space(1))) v4u32 *)p;
    return make_uint4(v.x, v.y, v.z, v.w);
}

/* ---- hit-run fast-forward helpers ------------------------------------------------------
 * A trace chunk is 8 packed instructions in 4 dwords (instruction j = half-word j).       */
/* 128-bit shifts on two 64-bit halves, branch-free (selects and 64-bit shifts only: a
 * select chain over a per-lane index is turned into divergent branches) */
DEVI void shr128(uint64_t &lo, uint64_t &hi, uint32_t b) {          /* b = 0..127 */
    const bool big = b >= 64u;
    const uint64_t l = big ? hi : lo, h = big ? 0ull : hi;
    const uint32_t c = b & 63u;
    lo = (l >> c) | ((h << 1) << (63u - c));
    hi = h >> c;
}
DEVI void shl128(uint64_t &lo, uint64_t &hi, uint32_t b) {          /* b = 0..128 */
    const bool big = b >= 64u, none = b >= 128u;
    const uint64_t h = big ? lo : hi, l = big ? 0ull : lo;
    const uint32_t c = b & 63u;
    hi = none ? 0ull : (h << c) | ((l >> 1) >> (63u - c));
    lo = none ? 0ull : l << c;
}
DEVI void to64(const uint32_t (&x)[4], uint64_t &lo, uint64_t &hi) {
    lo = x[0] | ((uint64_t)x[1] << 32);
    hi = x[2] | ((uint64_t)x[3] << 32);
}
DEVI void from64(uint64_t lo, uint64_t hi, uint32_t (&y)[4]) {
    y[0] = (uint32_t)lo; y[1] = (uint32_t)(lo >> 32); y[2] = (uint32_t)hi; y[3] = (uint32_t)(hi >> 32);
}
/* the 8 instructions starting at half-word s (0..7) of the 16 in (a, b): low 128 bits of
 * (b:a) >> 16 s */
DEVI void ff_window(const uint32_t (&a)[4], const uint32_t (&b)[4], uint32_t s, uint32_t (&w)[4]) {
    uint64_t al, ah, bl, bh;
    to64(a, al, ah);
    to64(b, bl, bh);
    shr128(al, ah, 16u * s);
    shl128(bl, bh, 128u - 16u * s);
    from64(al | bl, ah | bh, w);
}
/* x << 16 s (128 bits, zero fill), s = 0..8 */
DEVI void ff_unshift(const uint32_t (&x)[4], uint32_t s, uint32_t (&y)[4]) {
    uint64_t l, h;
    to64(x, l, h);
    shl128(l, h, 16u * s);
    from64(l, h, y);
}
/* x >> 16 s (128 bits, zero fill): the shift-register form of an aligned chunk at ip & 7 = s */
DEVI void ff_shift(const uint32_t (&x)[4], uint32_t s, uint32_t (&y)[4]) {
    uint64_t l, h;
    to64(x, l, h);
    shr128(l, h, 16u * s);
    from64(l, h, y);
}
/* GEN: aligned chunk c (instructions 8c .. 8c+7) of the counter-based generator, in the
 * packed-trace layout (gen_instr's key and bit fields) */
template <int NP>
DEVI void gen_chunk(uint64_t gmul, int dist, uint64_t sysg, uint32_t node, uint32_t c,
                    uint32_t (&w)[4]) {
#pragma unroll
    for (int half = 0; half < 2; ++half) {
        const uint32_t i0 = (c * 8u + 4u * half) & 0xFFFu;
        const uint64_t r = splitmix(gmul + ((sysg << 16) | ((uint64_t)node << 12) | (uint64_t)(i0 >> 2)));
#pragma unroll
        for (int j = 0; j < 2; ++j)
            w[2 * half + j] = instr_from_bits<NP>((uint32_t)(r >> (32 * j)) & 0xFFFFu, dist) |
                              (instr_from_bits<NP>((uint32_t)(r >> (32 * j + 16)) & 0xFFFFu, dist) << 16);
    }
}
/* minimum over the NP lanes of a node group (all of them active): DPP quad swaps, then the
 * half-row mirror for 8-lane groups */
template <int NP>
DEVI uint32_t gmin(uint32_t x) {
    uint32_t y = (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0xB1, 0xF, 0xF, false);
    x = y < x ? y : x;
    y = (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x4E, 0xF, 0xF, false);
    x = y < x ? y : x;
    if (NP == 8) {
        y = (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x141, 0xF, 0xF, false);
        x = y < x ? y : x;
    }
    return x;
}


/* ---- the transition kernel ------------------------------------------------------------ *
 * One loop iteration = one lock-step round of every system resident in the wave.  The 13
 * message handlers + 2 issue paths are ONE predicated data flow (shared decode, per-type
 * predicates, selects): a divergent 17-way switch costs every wave the sum of the taken
 * cases plus their exec-mask bookkeeping.  Only the once-per-node dump, the trace-chunk
 * refill and the per-system finish are real branches.                                   */
/* MODE bits: the optional parts of a round, compiled in only where asked for */
enum : int {
    M_TC = 1,   /* per-type message counters (DSM_F_TYPE_COUNTS): 16-bit fields per node and
                 * system, added to the wave counters when the system finishes             */
    M_TR = 2,   /* issue-order trace (DSM_F_ISSUE_TRACE): DEBUG_INSTR order, :595-598      */
    M_SX = 4,   /* seeded schedule exploration (dsm_set_schedule): a node with an action
                 * may stall for the round (oracle/dsm_common.h dsm_sched_act)            */
    M_LIM = 8,  /* run-time round limit / inbox limit (dsm_set_round_limit,
                 * dsm_set_inbox_limit) for the bench mode, which otherwise has them as
                 * constants (measured: the two limits as SGPRs cost 1.5-2% in the round)  */
    M_NOFF = 16,/* the bench mode without the hit-run fast-forward (ffscan_kernel picks)     */
    M_SERB = 32 /* with M_NOFF: the budget pass of a serial-resumed run (suspend-on-lone, the
                 * serial-form record); the plain budget pass of a fast-forward-resumed run
                 * is the kernel without them (measured on C4: 41.1 -> 40.0 ms per run)    */
};

/* ---- fast-forward verdict --------------------------------------------------------------
 * The hit-run fast-forward (sim_kernel step (0)) pays only where nodes issue long runs of
 * hits; elsewhere its second copy of the round costs the plain round ~3% (C3).  Before the
 * packed path's budget pass, ffscan_kernel replays the first instructions of a sample of
 * node traces through a private 4-line tag model (each line holds the last address that
 * mapped to it, assignment.c:177-184 indexing; no coherence) and counts the instructions
 * that end a run of 8 hits.  Both kernels of the pair are launched; the one this verdict
 * does not pick exits at once.  The choice only moves time: both produce the same results
 * (tests/test_gpu_fastforward.py). */
constexpr uint32_t SCAN_SYS = 4096, SCAN_INSTR = 256;
DEVI bool ff_verdict(const uint32_t *scan) {
    const uint32_t tot = scan[0], run8 = scan[1];
    return run8 != 0u && (uint64_t)run8 * 16u >= tot;    /* >= 1/16 of the sample */
}
template <int NP>
__global__ void __launch_bounds__(256) ffscan_kernel(const uint16_t *traces, const uint32_t *counts,
                                                     uint32_t stride, uint64_t n_sys, uint32_t *scan,
                                                     unsigned long long *counters) {
    const uint32_t S = n_sys < SCAN_SYS ? (uint32_t)n_sys : SCAN_SYS;
    const uint32_t t = blockIdx.x * 256u + threadIdx.x;
    uint32_t tot = 0, run8 = 0;
    if (t < S * NP) {
        const uint64_t sys = (uint64_t)(t / NP) * n_sys / S;
        const uint32_t node = t % NP;
        const uint32_t c = counts[sys * NP + node];
        const uint32_t n = (c < stride ? c : stride) < SCAN_INSTR ? (c < stride ? c : stride) : SCAN_INSTR;
        const uint16_t *tp = traces + (sys * NP + node) * (uint64_t)stride;
        uint32_t tags = 0xFFFFFFFFu, run = 0;
        for (uint32_t i = 0; i < n; i += 8) {
            const uint4 v = ld16(tp + i);
            const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                if (i + j < n) {
                    const uint32_t a = (w[j >> 1] >> (16 * (j & 1) + 8)) & 0x7Fu, sh = (a & 3u) * 8u;
                    run = ((tags >> sh) & 0xFFu) == a ? run + 1u : 0u;
                    tags = (tags & ~(0xFFu << sh)) | (a << sh);
                    run8 += run >= 8u ? 1u : 0u;
                }
            }
        }
        tot = n;
    }
    for (int o = 1; o < 64; o <<= 1) {
        tot += __shfl_xor(tot, o, 64);
        run8 += __shfl_xor(run8, o, 64);
    }
    if ((threadIdx.x & 63u) == 0 && tot) {
        atomicAdd(&scan[0], tot);
        atomicAdd(&scan[1], run8);
        atomicAdd(&counters[K_SCANI], (unsigned long long)tot);
        atomicAdd(&counters[K_SCANR], (unsigned long long)run8);
    }
}

template <int NP, int RING, int WAVES, bool GEN, int MODE, int OCC = 5>
__global__ void __launch_bounds__(64 * WAVES) __attribute__((amdgpu_waves_per_eu(OCC)))
sim_kernel(const SimArgs *Ap) {
    constexpr int GPW = 64 / NP;
    constexpr uint32_t NPM = (1u << NP) - 1u;
    constexpr bool FB = (RING == FB_RING);   /* the 256-deep re-run kernel                */
    constexpr bool TC = (MODE & M_TC) != 0, TR = (MODE & M_TR) != 0, SX = (MODE & M_SX) != 0;
    constexpr bool BUD = (MODE & ~(M_LIM | M_NOFF | M_SERB)) == 0 && !FB && !GEN;   /* two-pass schedule */
    constexpr bool LIM = FB || (MODE & ~(M_NOFF | M_SERB)) != 0;   /* limits read at run time, else constants */
    /* hit-run fast-forward: wherever the order of issues inside a round is not observed
     * (not with the issue-order trace or the seeded stalls of schedule exploration) */
    constexpr bool FF = (MODE & (M_TR | M_SX | M_NOFF)) == 0;
    /* suspend-on-lone and the serial-form record: the plain budget kernel of a serial-resumed
     * run only (M_SERB) */
    constexpr bool LONE = BUD && !FF && (MODE & M_SERB) != 0;
    constexpr bool UNI = SIM_UNI != 0 && LONE;     /* the per-round end test as one ballot */
    /* paired refills (SIM_R2): the plain kernels, whose ip only ever moves by one issue */
    constexpr bool R2 = SIM_R2 != 0 && BUD && !FF && !GEN;
    constexpr int SW = susp_words(RING);
    /* fast-forward probe interval: FF_PROBE iterations after a probe that found a group,
     * doubling up to FF_PROBE_MAX after each one that found none (workloads without hit
     * runs stop paying for the probe) */
    constexpr uint32_t FF_PROBE = 4, FF_PROBE_MAX = 512;

    /* one of a fast-forward / plain pair: the kernel the trace scan's verdict did not pick
     * exits at once (wave-uniform scalar loads; the whole workgroup returns before any
     * barrier).  A budget pass always runs on the plain one: its rounds are the cold start,
     * misses rather than hit runs, where the fast-forward step's probes only cost (C4: 48.2
     * -> 46.4 ms per step) */
    if (!FB && Ap->ffsel && (ff_verdict(Ap->scan) && !Ap->budget) != FF) return;
    /* ... and of the two plain budget kernels (SimArgs::split), the one for the resume pass
     * the verdict picked: M_SERB for the serial one, the other for the fast-forward one */
    if (!FB && !FF && Ap->split && Ap->budget && ff_verdict(Ap->scan) == LONE) return;

    __shared__ uint32_t s_mb[WAVES][8][64];          /* 2 x (mem | bv << 8) per dword */
    __shared__ uint32_t s_line[WAVES][4][64];        /* cache lines: addr | value << 8 | state << 16 */
    __shared__ uint32_t s_ring[WAVES][RING][64];                       /* inbox rings   */
    __shared__ __attribute__((aligned(16))) uint32_t s_out[WAVES][128]; /* 2 words/lane  */
    __shared__ uint32_t s_rm[WAVES][64];                               /* receive masks */
    __shared__ unsigned long long s_cnt[WAVES][K_N];
    __shared__ uint2 s_tab[DT_TABLE_WORDS / 2];                /* micro-op table + header */

    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint32_t node = lane % NP, gbase = lane - node;
    if (lane < K_N) s_cnt[wv][lane] = 0;
    s_rm[wv][lane] = 0;
    for (uint32_t i = threadIdx.x; i < DT_TABLE_WORDS / 2; i += 64 * WAVES) s_tab[i] = Ap->table[i];
    __syncthreads();
#if SIM_TAILPROBE
    const uint64_t tprobe0 = __builtin_amdgcn_s_memrealtime();
#endif

    /* values read through loaded (generic) pointers count as lane-varying to the compiler's
     * uniformity analysis, which then takes every branch that depends on them -- the round
     * loop's -- as divergent: SIM_RFL states them uniform */
    const uint64_t n = SIM_RFL ? uni64(Ap->d_n ? (uint64_t)*Ap->d_n : Ap->n_sys)
                               : (Ap->d_n ? (uint64_t)*Ap->d_n : Ap->n_sys);
    const bool ffv = SIM_RFL ? uni32(ff_verdict(Ap->scan)) != 0u : ff_verdict(Ap->scan);
    const uint32_t *list = Ap->list;
    const uint64_t G = ((uint64_t)blockIdx.x * WAVES + wv) * GPW + lane / NP;
    uint32_t shard = blockIdx.x & 7u, tried = 0;
    /* GEN: loop-invariant generator parameters */
    const uint64_t gmul = GEN ? Ap->seed * 0x9E3779B97F4A7C15ULL : 0;
    const uint64_t gfirst = GEN ? Ap->first_sys : 0;
    const int gdist = GEN ? Ap->dist : 0;
    const uint32_t stride = GEN ? 0u : Ap->stride;   /* >= 8, multiple of 8 (dsm_open) */
    const uint32_t lim_rsh = LIM ? Ap->lim_rsh : RSH_MAX;   /* round limit 1 << lim_rsh    */
    /* an inbox beyond ocap ends the round's system: the fast kernel hands it to the 256-deep
     * re-run (its ring holds RING), which reports RING_OVERFLOW beyond the inbox limit */
    const uint32_t ocap = FB || (LIM && Ap->icap < (uint32_t)RING) ? Ap->icap : (uint32_t)RING;
    const uint32_t rsh0 = BUD && Ap->rsh < lim_rsh ? Ap->rsh : lim_rsh;
    /* the round test's threshold: the round limit, or the budget pass's budget (wave-uniform) */
    uint32_t thr = 1u << rsh0;
    if (BUD && Ap->budget && Ap->thr_ff && (FF || (Ap->ffsel && ffv)) &&
        Ap->thr_ff < (1u << lim_rsh))
        thr = Ap->thr_ff;          /* a fast-forward workload's budget (thr_ff, run_engine) */
    const uint32_t late_rsh = BUD ? Ap->late_rsh : 0u;
    const bool budget = BUD && Ap->budget != 0, resume = BUD && Ap->resume != 0;
    /* suspend-on-lone: the budget pass of a run whose resume pass is the serial one (not the
     * fast-forward pair's pick) */
    const uint32_t lone_on = (LONE && budget && !(Ap->ffsel && ffv)) ? Ap->lone : 0u;
    uint32_t lcd = lone_on;             /* rounds to the next check (uniform) */
    const uint32_t lone_min = Ap->lone_min;   /* not before this many rounds */
    const bool ser_fmt = LONE && budget && Ap->serfmt && !(Ap->ffsel && ffv);
    /* systems started statically (one per slot), the rest claimed from the shard counters.
     * The resume pass is launched at the full grid and sizes itself here from the device-
     * resident count of suspended systems (no host round trip): it uses the fewest slots
     * that hold an equal whole number of them, so the slots (all running systems of similar
     * remaining length) finish together; the other slots exit at once. */
    auto pool_of = [&]() -> uint64_t {     /* recomputed where used (scalar registers are scarce) */
        uint64_t pool = (uint64_t)gridDim.x * WAVES * GPW;
        if (resume && n) {
            const uint64_t per = (n + pool - 1) / pool;
            pool = (n + per - 1) / per;
        }
        return pool;
    };

    Node nd;
    uint32_t cur[4] = {0, 0, 0, 0}, nxt[4] = {0, 0, 0, 0};
    /* R2: chunk k + 2 while the chunk in cur (k = ip >> 3) is even; the refill consuming an
     * odd chunk loads k + 2 and k + 3 together (one line fetch for both) */
    uint32_t nx2[4] = {0, 0, 0, 0};
    /* FF: the line tags for a hit, a byte per line (RD needs a valid line, state != I; WR one
     * in M or E, state <= E; 0xFF never equals a 7-bit address), set at mode entry: in the
     * mode no message arrives and a write hit on E leaves M, still a hit for both */
    uint32_t fkr = 0, fkw = 0;
    uint64_t sys = 0;
    /* this node's trace slot, set when a system starts (measured: recomputing it at each
     * refill costs more than the two VGPRs) */
    const uint16_t *const traces = Ap->traces;
    auto tslot = [&]() { return traces + (sys * NP + node) * (uint64_t)stride; };
    const uint16_t *tb = nullptr;
    uint32_t rounds = 0, rmsg = 0;
    bool live = false;
    uint32_t tc[7] = {0, 0, 0, 0, 0, 0, 0};                                  /* TC only */
    uint32_t nev = 0;                          /* TR: issue events of the system so far */
    const uint64_t smul = SX ? Ap->sched_seed * 0x9E3779B97F4A7C15ULL : 0;
    const uint32_t sthr = SX ? Ap->sched_thresh : 0;
    nd.dst = nd.ctl = nd.ip = nd.nins = nd.rh = nd.nmsg = 0;

    /* initializeProcessor :778-790 and main :142-146 for a new system in this lane's group */
    auto start = [&](uint64_t s) {
        /* the resume pass takes its list last-suspended first: those were cut short by the
         * late budget and may hold the most remaining rounds (measured: better than an
         * order by instructions left to issue, 85.0 vs 92.2 ms on C3) */
        sys = list ? (uint64_t)list[resume ? n - 1 - s : s] : s;
        if (resume) {                 /* continue a system the budget pass suspended */
            const uint32_t *sp = Ap->susp + sys * (uint64_t)(SW * NP) + node;
#pragma unroll
            for (int i = 0; i < 8; ++i) s_mb[wv][i][lane] = sp[i * NP];
#pragma unroll
            for (int i = 0; i < 4; ++i) s_line[wv][i][lane] = sp[(8 + i) * NP];
#pragma unroll
            for (int i = 0; i < RING; ++i) s_ring[wv][i][lane] = sp[(12 + i) * NP];
            const uint32_t *q = sp + (12 + RING) * NP;
            nd.dst = q[0]; nd.ctl = q[NP]; nd.ip = q[2 * NP]; nd.nins = q[3 * NP];
            nd.rh = q[4 * NP]; nd.nmsg = q[5 * NP]; rounds = q[6 * NP];
#pragma unroll
            for (int k = 0; k < 4; ++k) { cur[k] = q[(7 + k) * NP]; nxt[k] = q[(11 + k) * NP]; }
            if (!GEN) tb = tslot();
            if (R2 && ((nd.ip >> 3) & 1u) == 0u) {          /* the even phase needs k + 2 */
                const uint32_t pc = (nd.ip & ~7u) + 16u;
                const uint4 v2 = ld16(tb + (pc + 8u <= stride ? pc : stride - 8u));
                nx2[0] = v2.x; nx2[1] = v2.y; nx2[2] = v2.z; nx2[3] = v2.w;
                wait_vmcnt0();
            }
            rmsg = s_ring[wv][nd.rh & 0xFFu][lane];          /* the head, as the loop keeps it */
            return;
        }
        /* an opaque copy of the node id: keeps these per-system constants from being
         * hoisted out of the round loop, where they would only take registers */
        uint32_t nn = node;
        asm volatile("" : "+v"(nn));
#pragma unroll
        for (int i = 0; i < 8; ++i)
            s_mb[wv][i][lane] = ((20u * nn + 2 * i) & 0xFFu) | (((20u * nn + 2 * i + 1) & 0xFFu) << 16);
        nd.dst = 0xAAAAAAAAu;
#pragma unroll
        for (int i = 0; i < 4; ++i) s_line[wv][i][lane] = DSM_LINE_INIT;
        nd.ctl = 0; nd.ip = 0; nd.rh = 0; nd.nmsg = 0;
        rounds = 0;
        nev = 0;
        if (TC) {
#pragma unroll
            for (int k = 0; k < 7; ++k) tc[k] = 0;
        }
        if (GEN) {
            nd.nins = Ap->n_instr;
        } else {
            const uint32_t c = Ap->counts[sys * NP + node];
            nd.nins = c < stride ? c : stride;
            tb = tslot();
            /* both chunks unconditionally (in-slot), then drain them here, once per system:
             * the round loop's only vmcnt wait is then the refill rotation */
            const uint4 v0 = ld16(tb), v1 = ld16(tb + (stride > 8 ? 8 : 0));
            cur[0] = v0.x; cur[1] = v0.y; cur[2] = v0.z; cur[3] = v0.w;
            nxt[0] = v1.x; nxt[1] = v1.y; nxt[2] = v1.z; nxt[3] = v1.w;
            if (R2) {
                const uint4 v2 = ld16(tb + (stride > 16 ? 16 : stride - 8));
                nx2[0] = v2.x; nx2[1] = v2.y; nx2[2] = v2.z; nx2[3] = v2.w;
            }
            wait_vmcnt0();
        }
    };

    if (G < n && G < pool_of()) {
        live = true;
        start(G);
    } else {
        nd.ctl = C_WAIT | C_DUMPED;              /* a dead lane never acts (step (1)) */
    }

    uint32_t wrounds = 0;    /* loop iterations of this wave (uniform) */
    uint64_t ffm = 0;                  /* lanes in fast-forward mode (wave-uniform)          */
    uint32_t ffip = 0;                 /* FF: the node's instruction index when its group
                                        * entered fast-forward mode (ff_settle)               */
    uint64_t liveb = __ballot(live);
    /* hit-run fast-forward, deferred write-back.  While a group is in the mode only the line
     * tags and states decide its hits (RD: valid; WR: M or E, and a hit on E leaves M, which
     * is a hit for every later instruction too), so the fast-forward step only counts rounds
     * and instructions.  What the hits wrote -- each line's value and state M (:640-645) and
     * pendingWriteValue (:633) -- is applied when the group leaves the mode, before its next
     * normal round: the last write to each line within [ffip, ip) and the last write overall,
     * found by scanning the instructions back from ip (all of them hits).  Lanes with go. */
    auto ff_settle = [&](bool go) {
        /* lines 0-3 (only those in M or E at mode entry: a write hit needs one, so the other
         * lines were not written in the segment) and pending (bit 4) */
        const uint32_t wl = (((fkw & 0xFFu) != 0xFFu) ? 1u : 0u) | (((fkw & 0xFF00u) != 0xFF00u) ? 2u : 0u) |
                            (((fkw & 0xFF0000u) != 0xFF0000u) ? 4u : 0u) | (((fkw >> 24) != 0xFFu) ? 8u : 0u);
        uint32_t need = (go && nd.ip > ffip && wl) ? (0x10u | wl) : 0u;
        uint32_t i = nd.ip, lval = 0, wm = 0, pv = 0;
        while (__ballot(need != 0u)) {
            if (need) {
                const uint32_t c = (i - 1u) >> 3;                  /* chunk of instruction i-1 */
                uint32_t w[4];
                if (GEN) {
                    gen_chunk<NP>(gmul, gdist, gfirst + sys, node, c, w);
                } else {
                    const uint4 v = ld16(tb + 8u * c);
                    w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
                }
#pragma unroll
                for (int j = 7; j >= 0; --j) {                     /* newest first */
                    const uint32_t ix = 8u * c + (uint32_t)j;
                    const uint32_t h = (w[j >> 1] >> (16 * (j & 1))) & 0xFFFFu;
                    const bool wr = (ix < i) & (ix >= ffip) & ((h & 0x8000u) != 0u);
                    const uint32_t ln = (h >> 8) & 3u;
                    const bool tp = wr & ((need & 16u) != 0u), tl = wr & (((need >> ln) & 1u) != 0u);
                    pv = tp ? (h & 0xFFu) : pv;
                    const uint32_t sh = 8u * ln;
                    lval = tl ? ((lval & ~(0xFFu << sh)) | ((h & 0xFFu) << sh)) : lval;
                    wm |= tl ? (1u << ln) : 0u;
                    need &= ~((tp ? 16u : 0u) | (tl ? (1u << ln) : 0u));
                }
                i = 8u * c;
                need = i > ffip ? need : 0u;
            }
        }
        if (go && nd.ip > ffip) {
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if ((wm >> q) & 1u) {          /* value written, state MODIFIED (0) */
                    const uint32_t lw = s_line[wv][q][lane];
                    s_line[wv][q][lane] = (lw & 0xFFu) | (((lval >> (8 * q)) & 0xFFu) << 8);
                }
            /* the pending value of the last write (a node that issued no write keeps its own) */
            nd.ctl = wm ? ((nd.ctl & ~0xFFu) | pv) : nd.ctl;     /* any write also set a line */
        }
    };
    /* budget pass with a serial resume, every `lone` rounds: the groups that are quiet and
     * lone after a round's delivery -- every inbox empty, exactly one node neither waiting
     * nor dumped, with instructions left -- are suspended at that round's end, before the
     * lone node's next issue; the serial pass applies such a node's whole transactions at
     * once (dsm_serial.h ser_macro) where this kernel takes ~3 rounds of 8 lanes each.  Once
     * lone, a system stays lone (the replies its waiting nodes wait for can no longer come). */
    auto lone_mask = [&]() -> uint64_t {
        const bool may = (nd.ctl & (C_WAIT | C_DUMPED)) == 0u;
        const uint64_t qb = __ballot(nd.rh >= 256u);                        /* inbox non-empty */
        const uint64_t ib = __ballot(may);                                  /* may act          */
        const uint64_t pb = __ballot(may && nd.ip < nd.nins);                /* ... and issue    */
        const uint32_t fq = (uint32_t)(qb >> gbase) & NPM, fi = (uint32_t)(ib >> gbase) & NPM;
        const uint32_t fp = (uint32_t)(pb >> gbase) & NPM;
        return __ballot(live && fq == 0u && fi != 0u && (fi & (fi - 1u)) == 0u && fp == fi &&
                        rounds >= lone_min);
    };
    /* one lock-step round of every system of the wave; compiled twice: with the
     * fast-forward step and its gating (WFF, while some group of the wave is in
     * fast-forward mode) and without (the plain round the wave runs otherwise) */
    auto round = [&](auto wff) {
        constexpr bool WFF = FF && decltype(wff)::value;
            if (WFF) {
                /* ---- (0) hit-run fast-forward (exact) -------------------------------------- *
                 * When every inbox of a system is empty, nothing reaches any of its nodes until
                 * one of them issues an instruction that sends: each round is one more local hit
                 * per non-waiting node (RD hit :607-611, WR hit on M/E :635-645; a waiting node
                 * stays idle, :578-581).  A hit never changes which later instructions hit (only
                 * E -> M and values), so each issuing node's run of hits is fixed by its trace
                 * and its 4 line tags.  A group in fast-forward mode applies the next k rounds
                 * at once each iteration, k = the minimum run over its issuing nodes within their
                 * next 8 instructions: per node the last value written to each line (state M),
                 * pendingWriteValue (:633) and the instruction index, rounds += k.  A node with
                 * its trace done but not yet dumped, no issuing node, or the round limit bound
                 * k; at k < 8 the group leaves the mode and runs this iteration's round normally
                 * (the one that breaks the run).  The shift register cur / nxt keeps its meaning,
                 * so the mode has no state but the wave's lane mask. */
                const bool inff = __builtin_amdgcn_inverse_ballot_w64(ffm);
                if (lane == 0) s_cnt[wv][K_FFITER] += 1;     /* fast-forward steps of the wave */
                uint32_t k = 8;
                bool lng = false;          /* the group's step ran past the window (FF_LONG) */
                if (inff) {
                    const bool iss = (nd.ctl & C_WAIT) == 0u && nd.ip < nd.nins;
                    const bool dpend = (nd.ctl & (C_WAIT | C_DUMPED)) == 0u && nd.ip >= nd.nins;
                    /* the hit keys (fkr / fkw), fixed while the group is in the mode */
                    const uint32_t kr = fkr, kw = fkw;
                    const uint32_t s = nd.ip & 7u, m = 8u - s;
                    uint32_t W[4];
                    if (GEN) {
                        uint32_t A[4], B[4];
                        gen_chunk<NP>(gmul, gdist, gfirst + sys, node, nd.ip >> 3, A);
                        gen_chunk<NP>(gmul, gdist, gfirst + sys, node, (nd.ip >> 3) + 1, B);
                        ff_window(A, B, s, W);
                    } else {        /* the next 8: cur's m, then nxt's first s */
                        uint32_t T[4];
                        ff_unshift(nxt, m, T);
    #pragma unroll
                        for (int q = 0; q < 4; ++q) W[q] = cur[q] | T[q];
                    }
                    /* the first miss among the 8, 4 at a time: each instruction's high byte
                     * (WR << 7 | address) selects its line's tag byte from kw : kr by one byte
                     * permute; a non-zero byte of tag ^ address is a miss */
                    auto misses = [&](uint32_t w0, uint32_t w1) -> uint32_t {
                        const uint32_t hb = __builtin_amdgcn_perm(w1, w0, 0x07050301u);
                        const uint32_t sel = (hb & 0x03030303u) | ((hb >> 5) & 0x04040404u);
                        const uint32_t x = __builtin_amdgcn_perm(kw, kr, sel) ^ (hb & 0x7F7F7F7Fu);
                        return (((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;   /* bit 8j+7 */
                    };
                    const uint32_t ma = misses(W[0], W[1]), mb = misses(W[2], W[3]);
                    const uint32_t run = ma ? (uint32_t)__builtin_ctz(ma) >> 3
                                            : (mb ? 4u + ((uint32_t)__builtin_ctz(mb) >> 3) : 8u);
                    /* a group with no node issuing makes no progress here */
                    const bool gany = ((__ballot(iss) >> gbase) & NPM) != 0u;
                    uint32_t r = iss ? run : (dpend || !gany ? 0u : 8u);
                    if (iss && r > nd.nins - nd.ip) r = nd.nins - nd.ip;
                    /* the round limit and the budget (thr): the round that reaches it runs
                     * normally, so a group never finishes or is suspended in the mode */
                    const uint32_t rmax = rounds + 1u >= thr ? 0u : thr - 1u - rounds;
                    if (r > rmax) r = rmax;
                    k = gmin<NP>(r);
                    /* ---- the run past the window (FF_LONG) ---------------------------------
                     * a group whose issuing nodes all hit the whole window scans on, FF_LONG_U
                     * chunks per step straight from the trace, for the first miss of each node
                     * (or its trace end, or the group's round bound rmax); k = the group's
                     * minimum once every node has covered it.  The run applies at once, the
                     * group leaves the mode and the round that breaks the run follows in this
                     * iteration (C4 runs hundreds of hits per node between misses, where the
                     * 8-wide window took one loop iteration per 8). */
                    if (FF_LONG && __ballot(k == 8u)) {
                        /* chunks per scan step: generated chunks hide no latency and eight
                         * unrolled generator calls spilled the fused kernel (103 VGPRs) */
                        constexpr int LU = GEN ? 1 : FF_LONG_U;
                        lng = k == 8u;                                    /* group-uniform */
                        constexpr uint32_t INF = 0xFFFFFFFFu;
                        const uint32_t nl = nd.nins - nd.ip;
                        uint32_t found = iss ? (nl < rmax ? nl : rmax) : INF;
                        uint32_t cc = (nd.ip >> 3) + 1u;     /* its first unscanned positions */
                        bool go = lng;
                        auto chunks = [&](uint32_t c, uint32_t (&w)[LU][4]) {
    #pragma unroll
                            for (int u = 0; u < LU; ++u) {
                                if (GEN) {
                                    gen_chunk<NP>(gmul, gdist, gfirst + sys, node, c + u, w[u]);
                                } else {
                                    const uint32_t pc = (c + u) * 8u;
                                    const uint4 v = ld16(tb + (pc + 8u <= stride ? pc : stride - 8u));
                                    w[u][0] = v.x; w[u][1] = v.y; w[u][2] = v.z; w[u][3] = v.w;
                                }
                            }
                        };
                        while (__ballot(go)) {
                            if (go) {
                                if (iss) {
                                    uint32_t w[LU][4];
                                    chunks(cc, w);
    #pragma unroll
                                    for (int u = LU - 1; u >= 0; --u) {    /* the first miss wins */
                                        const uint32_t xa = misses(w[u][0], w[u][1]), xb = misses(w[u][2], w[u][3]);
                                        const uint32_t q = xa ? (uint32_t)__builtin_ctz(xa) >> 3
                                                              : (xb ? 4u + ((uint32_t)__builtin_ctz(xb) >> 3) : 8u);
                                        const uint32_t rel = 8u * (cc + u) + q - nd.ip;
                                        found = (q < 8u && rel < found) ? rel : found;
                                    }
                                }
                                /* every node's run is at least its coverage unless found */
                                const uint32_t gc = gmin<NP>(iss ? 8u * (cc + LU) - nd.ip : INF);
                                go = gmin<NP>(found) > gc;
                                cc += LU;
                            }
                        }
                        if (lng) k = gmin<NP>(found);
                    }
                    if (iss && k && lng) {
                        if (!GEN) {     /* the shift register at the new position */
                            const uint32_t ni = nd.ip + k, pc = (ni >> 3) * 8u;
                            const uint4 v0 = ld16(tb + (pc + 8u <= stride ? pc : stride - 8u));
                            const uint4 v1 = ld16(tb + (pc + 16u <= stride ? pc + 8u : stride - 8u));
                            const uint32_t X[4] = {v0.x, v0.y, v0.z, v0.w};
                            ff_shift(X, ni & 7u, cur);
                            nxt[0] = v1.x; nxt[1] = v1.y; nxt[2] = v1.z; nxt[3] = v1.w;
                        }
                        nd.ip += k;
                    } else if (iss && k) {
                        /* the write-back of the hits is deferred (ff_settle) */
                        if (!GEN) {     /* consume k from the shift register cur ++ nxt */
                            const bool cross = k >= m;
                            uint32_t X[4];
    #pragma unroll
                            for (int q = 0; q < 4; ++q) X[q] = cross ? nxt[q] : cur[q];
                            ff_shift(X, cross ? k - m : k, cur);
                            if (cross) {   /* the chunk after: used next iteration at the earliest */
                                const uint32_t pc = ((nd.ip >> 3) + 2) * 8u;
                                const uint4 v = ld16(tb + (pc + 8u <= stride ? pc : stride - 8u));
                                nxt[0] = v.x; nxt[1] = v.y; nxt[2] = v.z; nxt[3] = v.w;
                            }
                        }
                        nd.ip += k;
                    }
                    rounds += k;
                }
                const uint32_t adv = (uint32_t)__builtin_popcountll(__ballot(inff && node == 0u && k != 0u));
                if (lane == 0) s_cnt[wv][K_FFPASS] += adv;   /* system steps that advanced */
                /* those leave the mode and run this iteration's round normally, with their
                 * hits written back first */
                const uint64_t leave = __ballot(inff && (k < 8u || lng));
                ffm &= ~leave;
                if (leave) ff_settle(__builtin_amdgcn_inverse_ballot_w64(leave));
            }
            /* still in the mode: no round here (the lane's bit of the wave-uniform mask) */
            const bool inff = WFF && __builtin_amdgcn_inverse_ballot_w64(ffm);
            uint32_t op = OP_IDLE, o0 = 0, o1 = 0, nccv = nd.rh >> 8;
            bool stall = false;
            if (!WFF || (liveb & ~ffm) != 0) {
            /* ---- (1) this round's action, from state at the start of the round ---------- */
            /* A dead lane holds an empty inbox and C_WAIT | C_DUMPED, so it never acts.  One
             * compare gives "inbox empty and not waiting": the count sits at bits 8+ of rh, the
             * flags at bits 8-11 of ctl.  C_DUMPED there is harmless (a dumped node has issued
             * every instruction and dumps once), and so are C_OVF / C_ASSERT (their system ends
             * in the round that sets them).  A node in fast-forward mode has an empty inbox and
             * takes no action here. */
            const uint32_t cnt0 = nd.rh >> 8, head0 = nd.rh & 0xFFu;
            bool hasMsg = cnt0 != 0;                                          /* :158-169 */
            const bool canIssue = (nd.rh | nd.ctl) < 256u && !inff;           /* :578-581 */
            bool doIssue = canIssue && nd.ip < nd.nins;                       /* :590-592 */
            bool doDump = canIssue && nd.ip >= nd.nins;                       /* :688-697 */
            if (SX) {           /* a node with an action may stall this round (dsm_sched_act) */
                const bool avail = hasMsg || doIssue || doDump;
                const uint64_t key = (sys << 26) ^ ((uint64_t)(rounds + 1) << 3) ^ (uint64_t)node;
                const uint32_t h = (uint32_t)(splitmix(smul + key) >> 48);
                stall = avail && h >= sthr;
                hasMsg = hasMsg && !stall;
                doIssue = doIssue && !stall;
                doDump = doDump && !stall;
            }
            /* trace refill: when this round's issue takes the last instruction of `cur`, the
             * chunk after `nxt` is requested NOW and rotated in at the end of the round, so its
             * HBM latency overlaps this round's transition and delivery (a load consumed in the
             * same basic block stalls the whole wave on HBM). */
            const bool refill = !GEN && doIssue && ((nd.ip + 1) & 7u) == 0 && nd.ip + 1 < nd.nins;
            uint4 pf, pf2;
            if (R2 && SIM_R2 == 2) {
                /* the rotation consuming an odd chunk loads the next two, 32 B in one line:
                 * k + 2 straight into nx2 (dead in this phase), k + 3 into pf */
                if (refill && ((nd.ip + 1) & 15u) == 0u) {
                    const uint4 a2 = ld16(tb + (nd.ip + 9 < stride ? nd.ip + 9 : stride - 8));
                    pf = ld16(tb + (nd.ip + 17 < stride ? nd.ip + 17 : stride - 8));
                    nx2[0] = a2.x; nx2[1] = a2.y; nx2[2] = a2.z; nx2[3] = a2.w;
                }
            } else if (R2) {
                /* the rotation consuming an odd chunk loads the next two, 32 B in one line */
                if (refill && ((nd.ip + 1) & 15u) == 0u) {
                    pf = ld16(tb + (nd.ip + 9 < stride ? nd.ip + 9 : stride - 8));
                    pf2 = ld16(tb + (nd.ip + 17 < stride ? nd.ip + 17 : stride - 8));
                }
            } else if (refill) {
                pf = ld16(tb + (nd.ip + 9 < stride ? nd.ip + 9 : stride - 8));
            }
            const uint32_t headn = (head0 + 1 == (uint32_t)RING) ? 0u : head0 + 1;
            nd.rh = hasMsg ? (headn | ((cnt0 - 1) << 8)) : nd.rh;
            uint32_t w = rmsg;
            if (doIssue) {
                uint32_t ins;
                if (GEN) {
                    ins = gen_instr<NP>(gmul, gdist, gfirst + sys, node, nd.ip);
                } else {
                    /* `cur` is a 128-bit shift register: the next instruction is its low half-word */
                    ins = cur[0] & 0xFFFFu;
                    cur[0] = __builtin_amdgcn_alignbit(cur[1], cur[0], 16);
                    cur[1] = __builtin_amdgcn_alignbit(cur[2], cur[1], 16);
                    cur[2] = __builtin_amdgcn_alignbit(cur[3], cur[2], 16);
                    cur[3] >>= 16;
                }
                w = dt_issue_word(ins);                          /* message-word layout */
                if (TR) {                  /* the group's issues of this round, in node order */
                    const uint32_t g = (uint32_t)(__ballot(true) >> gbase) & NPM;
                    const uint32_t pos = nev + __builtin_popcount(g & ((1u << node) - 1u));
                    if (pos < Ap->issue_cap) Ap->issue[sys * Ap->issue_cap + pos] = (node << 16) | ins;
                }
                nd.ip++;
            }
            if (TR) nev += __builtin_popcount((uint32_t)(__ballot(doIssue) >> gbase) & NPM);
            op = (hasMsg || doIssue) ? dt_type(w) : doDump ? OP_DUMP : OP_IDLE;

            /* ---- (2) decode, then the micro-op table (dsm_table.h) ------------------------ */
            DtIn in;
            dt_decode(w, &in.a, &in.v, &in.excl, &in.r2, &in.s);
            const uint32_t blk = in.a & 15u, idx = in.a & 3u;                  /* :177-184 */
            uint16_t *const mbp = reinterpret_cast<uint16_t *>(&s_mb[wv][blk >> 1][lane]) + (blk & 1u);
            const uint32_t mbw = *mbp;
            in.op = op; in.node = node; in.np_mask = NPM;
            const uint32_t lw = s_line[wv][idx][lane];
            in.La = lw & 0xFFu; in.Lv = (lw >> 8) & 0xFFu; in.Ls = lw >> 16;
            in.Db = mbw >> 8; in.Ds = get2(nd.dst, blk); in.Mv = mbw & 0xFFu; in.pend = nd.ctl & 0xFFu;
            uint32_t evDb;
            /* header of op' = dt_opx(in): indexed by op | home << 5 (dt_build's second half
             * maps EVICT_SHARED at its home to DT_EVSH); with fewer than 8 nodes an instruction
             * whose home is not simulated is DT_ASSERT */
            uint32_t hix = op | ((in.a >> 4) == node ? 32u : 0u);
            if (NP < 8) hix = (op == DT_RD && (in.a >> 4) >= (uint32_t)NP) ? (uint32_t)DT_ASSERT : hix;
            const uint32_t hdr = reinterpret_cast<const uint32_t *>(&s_tab[DT_ENTRIES])[hix];
            const uint32_t ti = dt_index(in, hdr, &evDb);
            const uint2 E = s_tab[ti];
            /* dt_x / dt_y from the raw words: w = {v, a | x << 7, ..}, lw = {La, Lv, Ls, 0},
             * mbw = {Mv, Db}, ctl = {pending, ..} */
            const uint32_t X = __builtin_amdgcn_perm(lw, w, 0x05040001u) & ~0x80u;
            const uint32_t Y = __builtin_amdgcn_perm(mbw, nd.ctl, 0x0C050400u) | ((evDb & 0xFFu) << 24);
            const DtOut o = dt_apply_xy(in, X, Y, E.x, E.y, evDb);
            o0 = o.o0; o1 = o.o1;

            /* ---- (3) write back (idle lanes rewrite unchanged values) ------------------- */
            s_line[wv][idx][lane] = __builtin_amdgcn_perm(o.S, o.P, 0x0C040100u);   /* nLa nLv nLs */
            nd.dst = set2(nd.dst, blk, o.nDs);
            *mbp = (uint16_t)(o.nMv | (o.nDb << 8));
            nd.ctl = (nd.ctl & ~o.cclr) | o.cset;      /* wait, pendingWriteValue (:633), assert */
            const bool isMsg = op <= T_EVM;
            if (FB) nd.nmsg += isMsg ? 1u : 0u;     /* else messages received, counted at delivery */
            if (TC) {
                const uint32_t inc = isMsg ? (1u << ((op & 1u) * 16)) : 0u, q = op >> 1;
    #pragma unroll
                for (uint32_t k = 0; k < 7; ++k) tc[k] += (q == k) ? inc : 0u;
            }
            if (doDump) {                                                    /* :688-697 */
                nd.ctl |= C_DUMPED;               /* printProcessorState(threadId, node), :695 */
                if (!REC_PROBE) store_rec<WAVES>(Ap->recs + (sys * NP + node) * 8, nd, s_mb, s_line, wv, lane, 2u);
            }

            /* ---- (4) end-of-round delivery: ascending sender, then program order --------- */
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            /* the outbox holds ring entries: body | sender << 24 (the masks stay in o0 / o1) */
            reinterpret_cast<uint2 *>(s_out[wv])[lane] = make_uint2(dt_ring_entry(o0, node), dt_ring_entry(o1, node));
            /* receive masks, transposed at the sender: word j of this node sets bit 2*node + j of
             * every destination's mask (LDS atomic OR; a multicast INV visits its destinations in
             * a short loop), so a receiver reads its mask instead of gathering bits from the
             * group's destination bytes */
            {
                uint32_t m0 = o0 >> 24, m1 = o1 >> 24;
                const uint32_t b0 = 2 * node;
                const uint32_t bit0 = 1u << b0, bit1 = 2u << b0;
#if SIM_BF & 1
                /* each word's first destination without a branch: a lane with none ORs 0 into
                 * its own mask */
                atomicOr(&s_rm[wv][m0 ? gbase + __builtin_ctz(m0) : lane], m0 ? bit0 : 0u);
                atomicOr(&s_rm[wv][m1 ? gbase + __builtin_ctz(m1) : lane], m1 ? bit1 : 0u);
                m0 &= m0 - 1;
                m1 &= m1 - 1;
#else
                if (m0) { atomicOr(&s_rm[wv][gbase + __builtin_ctz(m0)], bit0); m0 &= m0 - 1; }
                if (m1) { atomicOr(&s_rm[wv][gbase + __builtin_ctz(m1)], bit1); m1 &= m1 - 1; }
#endif
                while (m0) { atomicOr(&s_rm[wv][gbase + __builtin_ctz(m0)], bit0); m0 &= m0 - 1; }
                while (m1) { atomicOr(&s_rm[wv][gbase + __builtin_ctz(m1)], bit1); m1 &= m1 - 1; }
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            uint32_t R = s_rm[wv][lane];     /* bit 2*sender+word: that word is addressed to me */
            s_rm[wv][lane] = 0;
            /* the fast kernel counts messages received (handled = received - still in the ring,
             * taken at the finish); an overflow is flagged here and set in ctl on the finish
             * path, where its system ends */
            if (!FB)      /* one v_bcnt with its accumulator (the compiler would share the count) */
                asm volatile("v_bcnt_u32_b32 %0, %1, %0" : "+v"(nd.nmsg) : "v"(R));
            {
                /* appended at the tail in R's bit order.  An overflowing ring sets C_OVF and its
                 * tail wraps onto live entries: the system ends this round (the transition
                 * kernel hands it to the 256-deep re-run, which reports RING_OVERFLOW), and the
                 * ring is not part of any record or result. */
                const uint32_t hh = nd.rh & 0xFFu, cc = nd.rh >> 8;
                const uint32_t ncc = cc + __builtin_popcount(R);
                nccv = ncc;
                uint32_t slot = hh + cc;
                slot = slot >= (uint32_t)RING ? slot - RING : slot;
                while (R) {
                    const uint32_t j = __builtin_ctz(R);
                    R &= R - 1;
                    s_ring[wv][slot][lane] = s_out[wv][2 * gbase + j];
                    slot = (slot + 1 == (uint32_t)RING) ? 0u : slot + 1;
                }
                nd.rh = hh | ((ncc < (uint32_t)RING ? ncc : (uint32_t)RING) << 8);
                rmsg = s_ring[wv][hh][lane];          /* next round's head, prefetched */
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            if (R2 && SIM_R2 == 2 && refill) {
                /* cur <- nxt <- nx2 always; after a pair load nx2 <- pf (k + 3) */
    #pragma unroll
                for (int k = 0; k < 4; ++k) { cur[k] = nxt[k]; nxt[k] = nx2[k]; }
                if ((nd.ip & 15u) == 0u) { nx2[0] = pf.x; nx2[1] = pf.y; nx2[2] = pf.z; nx2[3] = pf.w; }
            } else if (R2 && refill) {
                /* ip is already past the issue: an even ip means an odd chunk was consumed */
                const bool pair = (nd.ip & 15u) == 0u;
    #pragma unroll
                for (int k = 0; k < 4; ++k) cur[k] = nxt[k];
                nxt[0] = pair ? pf.x : nx2[0]; nxt[1] = pair ? pf.y : nx2[1];
                nxt[2] = pair ? pf.z : nx2[2]; nxt[3] = pair ? pf.w : nx2[3];
                if (pair) { nx2[0] = pf2.x; nx2[1] = pf2.y; nx2[2] = pf2.z; nx2[3] = pf2.w; }
            } else if (refill) {
    #pragma unroll
                for (int k = 0; k < 4; ++k) cur[k] = nxt[k];
                nxt[0] = pf.x; nxt[1] = pf.y; nxt[2] = pf.z; nxt[3] = pf.w;
            }

            }   /* normal round */

            /* ---- (5) per-system termination (Appendix A step 4) -------------------------- *
             * A round in which no node of a system acts changes nothing, so every later round
             * is idle too: the active rounds of a system are a prefix, and `rounds` counts every
             * round, less the final idle one.  The per-round test is wave-uniform: a live group
             * with no active lane (a zero field in actb | ~liveb), or a lane with an assert, an
             * overflow or the round limit; the per-lane finish runs only then.  A group in
             * fast-forward mode counted its rounds in step (4b) and is active. */
            if (!inff) ++rounds;
            /* both tests on VGPR integers (one compare each; the round limit is a power of two) */
            uint32_t opv = op;
            asm volatile("" : "+v"(opv));
            const uint64_t actb = __ballot(opv != OP_IDLE || stall) | (WFF ? ffm : 0ull);
            uint64_t loneb = 0;
            if (SIM_RFL) lcd = uni32(lcd);
            if (!WFF && LONE && lone_on && --lcd == 0u) {
                lcd = lone_on;
                loneb = lone_mask();
            }
            /* rounds >= thr: the round limit, or the budget pass's budget */
            if constexpr (UNI) {
                /* one ballot: a live lane whose group has no active lane (its field of actb), or
                 * with an assert, the round limit / budget or an overflowing inbox (C3 budget
                 * pass 24.5 -> 23.8 ms, C5 15.9 -> 15.5; in the kernel without suspend-on-lone,
                 * C4's, 17.3 -> 17.6: there the mask form below is kept) */
                uint32_t gidle;
                if constexpr (SIM_UNI == 2) {
                    /* the groups with an active lane as a wave mask, each such group's field
                     * all ones (scalar ops on the uniform actb), read per lane as a lane mask */
                    constexpr uint64_t FTOP = NP == 8 ? 0x8080808080808080ull : 0x8888888888888888ull;
                    constexpr uint64_t FLOW = ~FTOP;
                    const uint64_t one = ((((actb & FLOW) + FLOW) | actb) & FTOP) >> (NP - 1);
                    gidle = __builtin_amdgcn_inverse_ballot_w64((one << NP) - one) ? 0u : 1u;
                } else {
                    gidle = ((uint32_t)(actb >> gbase) & NPM) == 0u;
                }
                /* bitwise, not && / ||: short-circuit conditions are compiled into branches */
                const uint32_t endc = (uint32_t)live & (gidle | (uint32_t)((nd.ctl & C_ASSERT) != 0u) |
                                                        (uint32_t)(rounds >= thr) | (uint32_t)(nccv > ocap));
                const uint64_t endb = __ballot(endc != 0u) | loneb;
                if (endb == 0) return;
            } else {
                /* a group field of actb | ~liveb that is zero: a live group with no active lane */
                const uint64_t flagb = __ballot((nd.ctl & C_ASSERT) != 0u || rounds >= thr) |
                                       __ballot(nccv > ocap) | loneb;
                constexpr uint64_t GLO = NP == 8 ? 0x0101010101010101ull : 0x1111111111111111ull;
                constexpr uint64_t GHI = GLO << (NP - 1);
                const uint64_t t = actb | ~liveb;
                if ((((t - GLO) & ~t & GHI) | (flagb & liveb)) == 0) return;
            }
            if (nccv > ocap) nd.ctl |= C_OVF;
            const uint32_t gact = (uint32_t)(actb >> gbase) & NPM;
            const uint64_t badb = __ballot(live && (nd.ctl & (C_ASSERT | C_OVF)));
            const bool gbad = ((badb >> gbase) & NPM) != 0;
            if (gact == 0) --rounds;
            /* budget pass: a system still running after thr rounds is suspended */
            const bool lone = ((loneb >> lane) & 1ull) != 0ull;
            const bool susp = budget && gact != 0 && !gbad && (rounds >= thr || lone) && (rounds >> lim_rsh) == 0u;
            const bool done = live && (gact == 0 || gbad || (rounds >> lim_rsh) != 0u || susp);

            const uint64_t doneb = __ballot(done);
            if (doneb) {
                if (FF) ffm &= ~doneb;        /* the slot's next system starts normally */
                const uint64_t dumpb = __ballot((nd.ctl & C_DUMPED) != 0u);
                const uint64_t asrb = __ballot((nd.ctl & C_ASSERT) != 0u);
                if (done) {
                    const uint32_t dmask = (uint32_t)(dumpb >> gbase) & NPM;
                    const bool gasr = ((asrb >> gbase) & NPM) != 0;
                    uint32_t st;
                    if (gasr) st = DSM_ASSERT_FAILED;
                    else if (gbad) st = DSM_RING_OVERFLOW;
                    else if (gact == 0) st = (dmask == NPM) ? DSM_COMPLETED : DSM_DEADLOCKED;
                    else st = DSM_ROUND_LIMIT;
                    const bool handoff = !FB && (st == DSM_RING_OVERFLOW);
                    const uint32_t fl = ((nd.ctl & C_WAIT) ? 1u : 0u) | ((nd.ctl & C_DUMPED) ? 2u : 0u);
                    if (!handoff && !susp && !REC_PROBE) store_rec<WAVES>(Ap->recs + (sys * NP + node) * 8 + 4, nd, s_mb, s_line, wv, lane, fl);
                    if (susp && ser_fmt && TRAFFIC_PROBE < 2) {    /* the serial pass's record (ssusp_words) */
                        uint32_t *sp = Ap->susp + sys * (uint64_t)ssusp_words(RING);
                        uint4 *mb = reinterpret_cast<uint4 *>(sp + 8u * node);     /* S_MB + 8 n */
                        mb[0] = make_uint4(s_mb[wv][0][lane], s_mb[wv][1][lane], s_mb[wv][2][lane], s_mb[wv][3][lane]);
                        mb[1] = make_uint4(s_mb[wv][4][lane], s_mb[wv][5][lane], s_mb[wv][6][lane], s_mb[wv][7][lane]);
                        uint32_t la = 0, lv = 0, ls = 0;
    #pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            const uint32_t l = s_line[wv][i][lane];
                            la |= (l & 0xFFu) << (8 * i);
                            lv |= ((l >> 8) & 0xFFu) << (8 * i);
                            ls |= ((l >> 16) & 3u) << (2 * i);
                        }
                        sp[64 + node] = la;                                 /* S_LA */
                        sp[72 + node] = lv;                                 /* S_LV */
                        sp[80 + node] = nd.dst;                             /* S_DS */
                        sp[88 + node] = (nd.ctl & 0x3FFu) | (ls << 10) | (nd.ip << 18);   /* S_CT */
                        sp[96 + node] = nd.rh;
                        sp[104 + node] = nd.nins;
                        sp[112 + node] = nd.nmsg;
                        if (node == 0) sp[120] = rounds;
                        /* a lone system's node: its chunks (the group has one node that may act) */
                        const bool mine = lone && (nd.ctl & (C_WAIT | C_DUMPED)) == 0u;
                        if (mine) {
                            reinterpret_cast<uint4 *>(sp + 124)[0] = make_uint4(cur[0], cur[1], cur[2], cur[3]);
                            reinterpret_cast<uint4 *>(sp + 128)[0] = make_uint4(nxt[0], nxt[1], nxt[2], nxt[3]);
                            sp[121] = node | 0x100u;
                        } else if (node == 0 && !lone) {
                            sp[121] = 0u;
                        }
                        const uint32_t h0 = nd.rh & 0xFFu, c0 = nd.rh >> 8;
                        for (uint32_t j = 0; j < c0; ++j) {      /* queued messages, oldest first */
                            const uint32_t sl = h0 + j;
                            sp[SSUSP_HDR + node * RING + j] = s_ring[wv][sl >= (uint32_t)RING ? sl - RING : sl][lane];
                        }
                    } else if (susp) {        /* save the node for the resume pass (start()) */
                        uint32_t *sp = Ap->susp + sys * (uint64_t)(SW * NP) + node;
    #pragma unroll
                        for (int i = 0; i < 8; ++i) sp[i * NP] = s_mb[wv][i][lane];
    #pragma unroll
                        for (int i = 0; i < 4; ++i) sp[(8 + i) * NP] = s_line[wv][i][lane];
    #pragma unroll
                        for (int i = 0; i < RING; ++i) sp[(12 + i) * NP] = s_ring[wv][i][lane];
                        uint32_t *q = sp + (12 + RING) * NP;
                        q[0] = nd.dst; q[NP] = nd.ctl; q[2 * NP] = nd.ip; q[3 * NP] = nd.nins;
                        q[4 * NP] = nd.rh; q[5 * NP] = nd.nmsg; q[6 * NP] = rounds;
    #pragma unroll
                        for (int k = 0; k < 4; ++k) { q[(7 + k) * NP] = cur[k]; q[(11 + k) * NP] = nxt[k]; }
                    }
                    const uint32_t ins = gsum32<NP>(nd.ip), msgs = gsum32<NP>(nd.nmsg - (FB ? 0u : nd.rh >> 8));
                    /* the serial pass's claim order, longest first by class: a lone system whose
                     * lone node has SER_LONG or more instructions left (the one lane with
                     * any: a group sum), or one still running several nodes, is long */
                    uint32_t lrem = 0;
                    if (SER_LONG && LONE)
                        lrem = gsum32<NP>((lone && (nd.ctl & (C_WAIT | C_DUMPED)) == 0u) ? nd.nins - nd.ip : 0u);
                    uint32_t nlo = 0xFFFFFFFFu, nhi = 0xFFFFFFFFu;
                    if (node == 0) {
                        if (susp) {
                            if (SER_LONG && LONE && ser_fmt && (!lone || lrem >= (uint32_t)SER_LONG)) {
                                const uint32_t lp = atomicAdd(Ap->susp_long, 1u);
                                Ap->susp_list[Ap->susp_cap - 1u - lp] = (uint32_t)sys;
                            } else {
                                const uint32_t pos = atomicAdd(Ap->susp_count, 1u);
                                Ap->susp_list[pos] = (uint32_t)sys;
                            }
                            atomicAdd(&s_cnt[wv][K_RESUMED], 1ull);
                        } else if (handoff) {
                            const uint32_t pos = atomicAdd(Ap->ovf_count, 1u);
                            Ap->ovf_list[pos] = (uint32_t)sys;
                            atomicAdd(&s_cnt[wv][K_OVFRERUN], 1ull);
                        } else {
                            reinterpret_cast<uint4 *>(Ap->results)[2 * sys] =
                                make_uint4(st | (dmask << 8), rounds, msgs, ins);
                            if (TR) Ap->issue_n[sys] = nev;
                            atomicAdd(&s_cnt[wv][K_MSGS], (unsigned long long)msgs);
                            atomicAdd(&s_cnt[wv][K_INSTRS], (unsigned long long)ins);
                            atomicAdd(&s_cnt[wv][K_ROUNDS], (unsigned long long)rounds);
                            atomicAdd(&s_cnt[wv][K_SYSTEMS], 1ull);
                            atomicAdd(&s_cnt[wv][K_STATUS + st], 1ull);
                            atomicMax(&s_cnt[wv][K_MAXR], (unsigned long long)rounds);
                        }
                        /* next system: static first assignment, then 8 sharded counters */
                        const uint64_t pool = pool_of();
                        const uint64_t rs = n > pool ? (n - pool + 7) / 8 : 0;
                        while (tried < 8) {
                            const uint64_t lo = pool + (uint64_t)shard * rs;
                            const uint64_t len = (n > lo) ? ((n - lo) < rs ? (n - lo) : rs) : 0;
                            if (len) {
                                const uint32_t r = atomicAdd(&Ap->claim[shard * 32u], 1u);
                                if (r < len) {
                                    const uint64_t nl = lo + r;
                                    nlo = (uint32_t)nl; nhi = (uint32_t)(nl >> 32);
                                    break;
                                }
                            }
                            shard = (shard + 1) & 7u;
                            ++tried;
                        }
                    }
                    if (TC && !handoff) {
    #pragma unroll
                        for (uint32_t t = 0; t < DSM_NTYPES; ++t) {
                            const uint32_t c = (tc[t >> 1] >> ((t & 1u) * 16)) & 0xFFFFu;
                            if (c) atomicAdd(&s_cnt[wv][t], (unsigned long long)c);
                        }
                    }
                    nlo = __shfl(nlo, (int)gbase, 64);
                    nhi = __shfl(nhi, (int)gbase, 64);
                    const uint64_t nl = ((uint64_t)nhi << 32) | nlo;
                    if (nl != NO_SYS) {
                        start(nl);
                    } else {
                        live = false;
                        nd.rh = 0;
                        nd.ctl = C_WAIT | C_DUMPED;      /* never acts again (round step (1)) */
                    }
                }
            }
            const uint64_t nlive = SIM_RFL ? uni64(__ballot(live)) : __ballot(live);
            /* budget pass: once a slot of this wave found no new system, the wave's remaining
             * systems get the late budget, so the launch's tail is not a system claimed last
             * running its full budget at falling occupancy (the resume pass continues them) */
            if (budget && late_rsh && (liveb & ~nlive) && (1u << late_rsh) < thr) thr = 1u << late_rsh;
            liveb = nlive;
    };

    /* the wave alternates between two loops, each with its own copy of the round: the plain
     * one (no fast-forward code at all) and, while some group is in fast-forward mode, the
     * one with the fast-forward step (0).  Separate inner loops keep the plain loop's
     * register allocation and code as if fast-forward did not exist. */
    uint32_t pint = FF_PROBE, pcd = FF_PROBE;   /* probe interval / countdown (uniform) */
    auto probe = [&]() {
        /* a group enters fast-forward mode when its inboxes are all empty, no node is about
         * to dump, and the next instruction of every issuing node (one at least) is a hit.
         * Only every so many iterations, so the round itself carries no detection work.
         * The lanes of a group are a field of the wave masks (8 bits for 8 nodes, 4 for 4);
         * a field's top bit is set iff the field is non-zero, then spread over it. */
        constexpr uint64_t FTOP = NP == 8 ? 0x8080808080808080ull : 0x8888888888888888ull;
        constexpr uint64_t FLOW = ~FTOP;
        const bool waits = (nd.ctl & C_WAIT) != 0u;
        const bool iss = !waits && nd.ip < nd.nins;
        bool hit = false;
        if (iss) {
            const uint32_t ins = GEN ? gen_instr<NP>(gmul, gdist, gfirst + sys, node, nd.ip)
                                     : (cur[0] & 0xFFFFu);
            const uint32_t a = (ins >> 8) & 0x7Fu;
            const uint32_t lw = s_line[wv][a & 3u][lane];
            const uint32_t ls = lw >> 16;
            hit = (lw & 0xFFu) == a && ((ins & 0x8000u) ? ls <= DT_CE : ls != DT_CI);
        }
        const bool block = (nd.rh >> 8) != 0u || (iss && !hit) ||
                           (!waits && !iss && (nd.ctl & C_DUMPED) == 0u);
        const uint64_t hitb = __ballot(hit);
        const uint64_t nzh = (((hitb & FLOW) + FLOW) | hitb) & FTOP;
        const uint64_t busy = __ballot(block) | ~liveb;
        const uint64_t nzb = (((busy & FLOW) + FLOW) | busy) & FTOP;
        const uint64_t one = (~nzb & nzh) >> (NP - 1);
        const uint64_t enter = ((one << NP) - one) & ~ffm;
        ffm |= enter;
        ffip = __builtin_amdgcn_inverse_ballot_w64(enter) ? nd.ip : ffip;   /* segment start */
        if (__builtin_amdgcn_inverse_ballot_w64(enter)) {
            const uint32_t L0 = s_line[wv][0][lane], L1 = s_line[wv][1][lane];
            const uint32_t L2 = s_line[wv][2][lane], L3 = s_line[wv][3][lane];
            const uint32_t la4 = __builtin_amdgcn_perm(L1, L0, 0x0C0C0400u) | __builtin_amdgcn_perm(L3, L2, 0x04000C0Cu);
            const uint32_t ls4 = __builtin_amdgcn_perm(L1, L0, 0x0C0C0602u) | __builtin_amdgcn_perm(L3, L2, 0x06020C0Cu);
            const uint32_t s_or_i = (ls4 >> 1) & 0x01010101u, inv = ls4 & s_or_i;
            fkr = la4 | ((inv << 8) - inv);
            fkw = la4 | ((s_or_i << 8) - s_or_i);
        }
        pint = one ? FF_PROBE : (pint < FF_PROBE_MAX ? 2u * pint : FF_PROBE_MAX);
        pcd = pint;
    };
    for (;;) {
        for (;;) {                                       /* plain rounds */
            if (liveb == 0) break;
            ++wrounds;
            if (FF && --pcd == 0u) {
                probe();
                if (ffm) break;
            }
            round(std::false_type{});
        }
        if (!FF || liveb == 0) break;
        for (;;) {                                       /* rounds with fast-forward */
            round(std::true_type{});
            if (ffm == 0 || liveb == 0) break;
            ++wrounds;
            if (--pcd == 0u) probe();
        }
    }

    /* publish the workgroup's counters: its waves' rows summed in LDS, then one device-scope
     * atomic per non-zero counter (integer sums mod 2^64 and a max: the result does not
     * depend on the order, so no separate reduction pass is needed) */
    if (lane == 0) {
        s_cnt[wv][K_WROUNDS] = wrounds;
#if SIM_TAILPROBE == 1
        /* probe build (results exact, not the default): when the budget pass's waves end, a
         * histogram in the msgs_by_type slots -- 0: before 14 ms, k = 1..11: [13 + k, 14 + k)
         * ms, 12: the waves' summed lifetimes in 10-ns ticks (s_memrealtime, 100 MHz) */
        if (BUD && budget) {
            const uint64_t dt = __builtin_amdgcn_s_memrealtime() - tprobe0;
            const uint64_t ms = dt / 100000u;
            s_cnt[wv][ms < 14u ? 0u : (ms - 13u < 11u ? ms - 13u : 11u)] += 1;
            s_cnt[wv][12] += dt;
        }
#endif
    }
    __syncthreads();
    if (threadIdx.x < K_N) {
        unsigned long long v = s_cnt[0][threadIdx.x];
#pragma unroll
        for (int w = 1; w < WAVES; ++w) {
            const unsigned long long x = s_cnt[w][threadIdx.x];
            v = threadIdx.x == K_MAXR ? (x > v ? x : v) : v + x;
        }
        if (v) {
            if (threadIdx.x == K_MAXR) atomicMax(&Ap->counters[K_MAXR], v);
            else atomicAdd(&Ap->counters[threadIdx.x], v);
        }
    }
}

/* ---- resume pass, serial form ------------------------------------------------------------
 * One lane = one suspended system, taken one node-action per iteration (dsm_serial.h): after
 * the budget pass the systems still running are almost all one surviving node issuing its
 * trace while the others wait for good, ~1.3 node-actions per round, so the lock-step
 * kernel's 8 lanes per system would idle ~84% of the time.  The state of 64 systems sits in
 * LDS as one column per lane ([word][lane]: every access is conflict-free and private to
 * its lane, so no barrier or fence is needed); a system's column is 104 words, so 6 waves
 * (26 KB each) fill the CU's 160 KB -- two waves on two of the four SIMDs, where round 2's
 * 153-word column allowed one per SIMD and nothing hid the iteration's dependent chain.
 * Each lane takes systems from the suspended list (last-suspended first), restores the
 * lock-step state (every inbox into the system's 8-slot queue, continued in the lane's spill
 * FIFO in HBM), runs it to the end and writes its result and final records; only an inbox
 * beyond the inbox limit hands the system to the 256-deep re-run, as a ring overflow of the
 * lock-step kernel does.  The issuing node's trace chunk and the next one are kept in
 * registers (refill step below). */
#ifndef SER_RF_DEF
#define SER_RF_DEF 8
#endif
#ifndef SER_GE_DEF
#define SER_GE_DEF 1
#endif
#ifndef SER_MACRO_DEF
#define SER_MACRO_DEF 1     /* lone-node macro-steps per iteration (0: off) */
#endif
/* SER_RF: iterations between trace refills; SER_GE: the one-action step (ser_step) runs in
 * every SER_GE-th iteration (the macro-step in every one) */
constexpr int SER_WAVES = 6, SER_RF = SER_RF_DEF, SER_GE = SER_GE_DEF;
constexpr int SER_MACRO = SER_MACRO_DEF;   /* lone-node macro-steps per iteration */
/* SER_PROBE builds (diagnostics, never the default): per-wave event counts of the serial pass
 * in the counter slots the pass leaves unused (msgs_by_type 0-4): iterations, iterations with
 * a macro-step, with a one-action step, with a chunk miss, hand-overs */
#ifndef SER_PROBE
#define SER_PROBE 0
#endif
#ifndef SER_HB
#define SER_HB 8            /* finished lanes that trigger a batched hand-over (1: at once) */
#endif
#ifndef SER_HT
#define SER_HT 32           /* ... or iterations the oldest finished lane has waited */
#endif

template <int W>
struct LdsCol {
    uint32_t (&s)[W][dsms::S_WORDS][64];
    uint32_t *dum;                        /* write-only dummy word of this lane              */
    uint32_t wv, lane;
    GU32 *sp;                             /* this lane's spill FIFO, S_SPILL words          */
    DEVI uint32_t ld(uint32_t w) const { return s[wv][w][lane]; }
    DEVI void st(uint32_t w, uint32_t v) const { s[wv][w][lane] = v; }
    /* a store when en, else to the dummy word: an address select, not a branch */
    DEVI void st_if(bool en, uint32_t w, uint32_t v) const { *(en ? &s[wv][w][lane] : dum) = v; }
    DEVI uint32_t ld8(uint32_t w, uint32_t b) const {
        return reinterpret_cast<const uint8_t *>(&s[wv][w][lane])[b];
    }
    DEVI void st8(uint32_t w, uint32_t b, uint32_t v) const {
        reinterpret_cast<uint8_t *>(&s[wv][w][lane])[b] = (uint8_t)v;
    }
    DEVI uint32_t ld16(uint32_t w, uint32_t h) const {
        return reinterpret_cast<const uint16_t *>(&s[wv][w][lane])[h];
    }
    DEVI void st16(uint32_t w, uint32_t h, uint32_t v) const {
        reinterpret_cast<uint16_t *>(&s[wv][w][lane])[h] = (uint16_t)v;
    }
    DEVI uint32_t sp_ld(uint32_t i) const { return sp[i]; }
    DEVI void sp_st(uint32_t i, uint32_t v) const { sp[i] = v; }
};
struct LdsTab {
    const uint2 (&t)[DT_TABLE_WORDS / 2];
    DEVI uint32_t hdr(uint32_t i) const { return reinterpret_cast<const uint32_t *>(&t[DT_ENTRIES])[i]; }
    DEVI void row(uint32_t i, uint32_t &w0, uint32_t &w1) const {
        const uint2 e = t[i];
        w0 = e.x;
        w1 = e.y;
    }
};

template <int NP, bool CAP>
__global__ void __launch_bounds__(64 * SER_WAVES) __attribute__((amdgpu_waves_per_eu(2)))
ser_kernel(const SimArgs *Ap) {
    using namespace dsms;
    constexpr uint32_t NPM = (1u << NP) - 1u;
    /* one of a fast-forward / serial pair: the fast-forward lock-step resume takes the run
     * when the trace scan picked fast-forward */
    if (Ap->ffsel && ff_verdict(Ap->scan)) return;

    __shared__ uint32_t s_ser[SER_WAVES][S_WORDS][64];
    __shared__ uint2 s_tab[DT_TABLE_WORDS / 2];
    __shared__ unsigned long long s_cnt[K_N];          /* the workgroup's counters */
    __shared__ uint32_t s_dum[64];                     /* dummy words (write-only)  */
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    if (threadIdx.x < K_N) s_cnt[threadIdx.x] = 0;
    for (uint32_t i = threadIdx.x; i < DT_TABLE_WORDS / 2; i += 64 * SER_WAVES) s_tab[i] = Ap->table[i];
    __syncthreads();
#if SIM_TAILPROBE
    const uint64_t tprobe0 = __builtin_amdgcn_s_memrealtime();
#endif

    const LdsCol<SER_WAVES> m{s_ser, &s_dum[lane], wv, lane,
                              (GU32 *)(Ap->spill + ((uint64_t)blockIdx.x * (64 * SER_WAVES) + threadIdx.x) * S_SPILL)};
    const LdsTab T{s_tab};
    /* claim k -> system: the long class first (SER_LONG: listed from the top down by the
     * budget pass, taken in suspension order), then the rest last-suspended first, as the
     * lock-step resume (their records the likeliest still in the MALL) */
    const uint32_t nlong = (SER_LONG && Ap->serfmt && Ap->susp_long) ? *Ap->susp_long : 0u;
    const uint32_t n = SIM_RFL ? uni32(*Ap->d_n + nlong) : *Ap->d_n + nlong;   /* (sim_kernel's n) */
    const uint32_t lcap = Ap->susp_cap;
    const uint32_t *const list = Ap->list;
    /* global (not flat) accesses: a pending flat operation makes every later wait a full
     * vmcnt(0) lgkmcnt(0), the LDS waits of the macro-step included */
    auto sel = [&](uint32_t k) -> uint32_t {
        return ((const GU32 *)list)[k < nlong ? lcap - 1u - k : n - 1u - k];
    };

    const uint32_t stride = Ap->stride, lim_rsh = Ap->lim_rsh, SR = Ap->susp_ring;
    const uint32_t cap = Ap->icap;
    const uint16_t *const traces = Ap->traces;

    /* uniform pointers, hoisted */
    uint4 *const recs = Ap->recs;
    dsm_sys_result *const results = Ap->results;
    const uint32_t *const susp = Ap->susp;
    uint32_t *const ovf_list = Ap->ovf_list;
    unsigned int *const ovf_count = Ap->ovf_count, *const claim_ctr = Ap->claim;

    SReg r;
    SCache cc;                      /* the lone node's words between macro-steps */
    ser_cache_clear(cc);
    uint64_t sys = 0;
    /* trace chunks of the node that issues (one at a time, almost always the same node):
     * cur = chunk tci of node tn, nx = chunk tci + 1 when nxv, pf = chunk pfc in flight.
     * Every prefetch is issued in the refill step that runs every SER_RF iterations and is
     * taken into nx at a later one, so a wait on it (the compiler's vmcnt(0)) only ever
     * covers loads issued SER_RF iterations earlier: a lane that rotates a chunk does not
     * stall the wave on HBM (measured: SER_RF 4 -> 16, 85.2 -> 82.7 ms on C3). */
    uint32_t tn = 0xFFu, tci = 0, pfc = 0;
    bool nxv = false, pfv = false;
    uint4 cur = make_uint4(0, 0, 0, 0), nx = cur, pf = cur;
    auto slot_of = [&](uint32_t nd) { return traces + (sys * NP + nd) * (uint64_t)stride; };

    auto claim_next = [&]() -> uint32_t {
        return gatomic_add((GU32 *)claim_ctr, 1u);
    };


    /* the state the budget pass suspended, in serial form (ssusp_words): the LDS column as
     * it is, in 16-byte row loads (two batches of 12, all in flight at once), then the
     * per-node header -- ring position, trace length, messages received -- and each
     * inbox's queued messages appended to the system's queue node by node (only each
     * inbox's own order matters; a lone system has none) */
    /* the same from the lock-step layout ([word][node], susp_words: a budget pass that ran
     * in the fast-forward kernel of a run with limits, M_LIM): memory / bitVector words as
     * they are, cache lines (addr | value << 8 | state << 16) split into the address, value
     * and control words */
    auto start_ls = [&]() {
        const GU32 *sp = (const GU32 *)(susp + sys * ((uint64_t)susp_words((int)SR) * NP));
        r.rounds = sp[(12u + SR + 6u) * NP];
        for (uint32_t nd = 0; nd < (uint32_t)NP; ++nd) {
            const GU32 *b = sp + nd;
#pragma unroll
            for (uint32_t i = 0; i < 8; ++i) m.st(S_MB + 8u * nd + i, b[i * NP]);
            uint32_t la = 0, lv = 0, ls = 0;
#pragma unroll
            for (uint32_t i = 0; i < 4; ++i) {
                const uint32_t l = b[(8u + i) * NP];
                la |= (l & 0xFFu) << (8 * i);
                lv |= ((l >> 8) & 0xFFu) << (8 * i);
                ls |= ((l >> 16) & 3u) << (2 * i);
            }
            m.st(S_LA + nd, la);
            m.st(S_LV + nd, lv);
            const GU32 *q = b + (12u + SR) * NP;
            const uint32_t ctl = q[NP], ip = q[2 * NP], rh = q[4 * NP];
            m.st(S_DS + nd, q[0]);
            m.st(S_CT + nd, (ctl & 0x3FFu) | (ls << SC_LS) | (ip << SC_IP));
            s_set_ni(r, nd, q[3 * NP]);
            const uint32_t h = rh & 0xFFu, c = rh >> 8;
            for (uint32_t j = 0; j < c; ++j) {
                uint32_t sl = h + j;
                sl = sl >= SR ? sl - SR : sl;
                ser_enqueue<S_QN>(m, r, nd, b[(12u + sl) * NP]);   /* <= 8 x 16: fits */
            }
            s_byte_add(r.cnt0, r.cnt1, nd, c);
            r.nz |= (c ? 1u : 0u) << nd;
            r.msgs += q[5 * NP] - c;       /* received - still queued = handled */
            r.iss |= ((ctl & (C_WAIT | C_DUMPED)) == 0u ? 1u : 0u) << nd;
            r.dmp |= ((ctl & C_DUMPED) ? 1u : 0u) << nd;
        }
    };
    const bool serfmt = Ap->serfmt != 0u;   /* the format the budget pass wrote */
    /* a serial-form record's 33 rows: the column (24) and the header (9), all in flight at
     * once; issued before the finished system's record stores at a hand-over, so that the
     * wait for them does not also wait for those stores (vmcnt counts both) */
    v4u32 rr[33];
    auto load_rec = [&](uint64_t s_) {
        const GV4 *sv = (const GV4 *)(susp + s_ * (uint64_t)ssusp_words((int)SR));
#pragma unroll
        for (uint32_t i = 0; i < 33; ++i) rr[i] = sv[i];
    };
    /* start the system `sys` (its rows in rr when the budget pass wrote the serial form) */
    auto start = [&]() -> uint32_t {
        ser_clear(r);
        tn = 0xFFu;                         /* the fetch cache: empty */
        nxv = pfv = false;
        if (!serfmt) {
            start_ls();
        } else {
        const GU32 *sp = (const GU32 *)(susp + sys * (uint64_t)ssusp_words((int)SR));
#pragma unroll
        for (uint32_t i = 0; i < 24; ++i) {
            const uint32_t w = 4u * i;
            m.st(w, rr[i].x); m.st(w + 1u, rr[i].y); m.st(w + 2u, rr[i].z); m.st(w + 3u, rr[i].w);
        }
        const v4u32 *const hd = rr + 24;
        r.rounds = hd[6].x;
        auto hw = [&](uint32_t k) -> uint32_t {        /* header word 96 + k, k < 24 (unrolled) */
            const v4u32 &v = hd[k >> 2];
            return (k & 3u) == 0u ? v.x : (k & 3u) == 1u ? v.y : (k & 3u) == 2u ? v.z : v.w;
        };
#pragma unroll
        for (uint32_t nd = 0; nd < (uint32_t)NP; ++nd) {
            const uint32_t rh = hw(nd), c = rh >> 8, ctl = m.ld(S_CT + nd);
            s_set_ni(r, nd, hw(8u + nd));
            for (uint32_t j = 0; j < c; ++j)
                ser_enqueue<S_QN>(m, r, nd, sp[SSUSP_HDR + nd * SR + j]);   /* <= 8 x 16: fits */
            s_byte_add(r.cnt0, r.cnt1, nd, c);
            r.nz |= (c ? 1u : 0u) << nd;
            r.msgs += hw(16u + nd) - c;    /* received - still queued = handled */
            r.iss |= ((ctl & (SC_WAIT | SC_DUMPED)) == 0u ? 1u : 0u) << nd;
            r.dmp |= ((ctl & SC_DUMPED) ? 1u : 0u) << nd;
        }
        /* a lone system: its node's chunks into the fetch cache, the shift register re-aligned
         * (instruction i of the chunk at half-word i; the consumed ones before ip read as 0) */
        if (hd[6].y & 0x100u) {
            tn = hd[6].y & 0xFFu;
            const uint32_t ip0 = m.ld(S_CT + tn) >> SC_IP, j0 = ip0 & 7u;
            const uint32_t rw[4] = {hd[7].x, hd[7].y, hd[7].z, hd[7].w};
            uint32_t al[4] = {0u, 0u, 0u, 0u};
#pragma unroll
            for (uint32_t k = 0; k < 8u; ++k) {        /* aligned half k = raw half k - j0 */
                uint32_t hv = 0u;
#pragma unroll
                for (uint32_t q = 0; q < 8u; ++q)
                    hv = (k >= j0 && k - j0 == q) ? ((rw[q >> 1] >> (16u * (q & 1u))) & 0xFFFFu) : hv;
                al[k >> 1] |= hv << (16u * (k & 1u));
            }
            cur = make_uint4(al[0], al[1], al[2], al[3]);
            nx = make_uint4(hd[8].x, hd[8].y, hd[8].z, hd[8].w);
            tci = ip0 >> 3;
            nxv = true;
            pfc = tci + 2u;                /* and the chunk after, in flight */
            pfv = pfc * 8u < stride;
            if (pfv) pf = ld16(slot_of(tn) + pfc * 8u);
        }
        }
        r.E = r.nz;
        r.A = r.nz | r.iss;
        ser_cache_clear(cc);
        if (r.A == 0u) {
            r.st = (r.dmp == NPM) ? SS_COMPLETED : SS_DEADLOCKED;
            return SR_DONE;
        }
        return SR_RUN;
    };
    auto store_rec = [&](uint32_t nd, uint32_t flags, uint32_t which) {
        if (REC_PROBE) return;
        GV4 *dst = (GV4 *)(recs + (sys * NP + nd) * 8 + 4u * which);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            v4u32 x;
            x.x = ser_rec_word(m, nd, flags, 4 * q);
            x.y = ser_rec_word(m, nd, flags, 4 * q + 1);
            x.z = ser_rec_word(m, nd, flags, 4 * q + 2);
            x.w = ser_rec_word(m, nd, flags, 4 * q + 3);
            dst[q] = x;
        }
    };
    auto fetch = [&](uint32_t nd, uint32_t ip, bool iss) -> uint32_t {
        /* bitwise & | on the flags: && / || chains are compiled into branches */
        const uint32_t c = ip >> 3;
        const bool tnd = tn == nd;
        const bool rot = iss & tnd & (tci + 1u == c) & nxv;              /* next chunk: in nx */
        const bool miss = iss & !rot & (!tnd | (tci != c));
        cur.x = rot ? nx.x : cur.x; cur.y = rot ? nx.y : cur.y;
        cur.z = rot ? nx.z : cur.z; cur.w = rot ? nx.w : cur.w;
        nxv = nxv & !rot;
        tci = rot ? c : tci;
        if (__ballot(miss)) {            /* another node issues, or a system's first issue */
            if (SER_PROBE && lane == 0) atomicAdd(&s_cnt[3], 1ull);
            if (miss) {       /* the chunk and the next one, both waited for here */
                const uint16_t *sl = slot_of(nd);
                cur = ld16(sl + 8u * c);
                nxv = (c + 1u) * 8u < stride;
                nx = ld16(sl + (nxv ? 8u * (c + 1u) : 8u * c));
                pfv = false;
                tn = nd;
                tci = c;
            }
            /* wait here, in the rare branch: left to the first use after the join, the wait
             * (vmcnt(0)) lands on the main path and also waits for the refill's prefetches */
            wait_vmcnt0();
        }
        /* word (ip & 7) / 2 of cur by masks: a select chain on a run-time index is turned
         * into a stack copy and an indexed scratch load */
        const uint32_t j = ip & 7u;
        const uint32_t m2 = 0u - ((j >> 1) & 1u), m4 = 0u - ((j >> 2) & 1u);
        const uint32_t lo = (cur.x & ~m2) | (cur.y & m2), hi = (cur.z & ~m2) | (cur.w & m2);
        const uint32_t wd = (lo & ~m4) | (hi & m4);
        return (wd >> (16u * (j & 1u))) & 0xFFFFu;
    };
    /* the macro-step's fetch: only from the chunks held in registers (cur, or nx by a
     * rotation), never a load -- a load here would put its wait (vmcnt(0)) on the main path,
     * where it also waits for the refill's prefetches and the record stores */
    auto fetch_reg = [&](uint32_t nd, uint32_t ip, uint32_t &ins) -> bool {
        const uint32_t c = ip >> 3;
        const bool tnd = tn == nd;
        const bool rot = tnd & (tci + 1u == c) & nxv;
        const bool have = tnd & ((tci == c) | rot);
        cur.x = rot ? nx.x : cur.x; cur.y = rot ? nx.y : cur.y;
        cur.z = rot ? nx.z : cur.z; cur.w = rot ? nx.w : cur.w;
        nxv = nxv & !rot;
        tci = rot ? c : tci;
        const uint32_t j = ip & 7u;
        const uint32_t m2 = 0u - ((j >> 1) & 1u), m4 = 0u - ((j >> 2) & 1u);
        const uint32_t lo = (cur.x & ~m2) | (cur.y & m2), hi = (cur.z & ~m2) | (cur.w & m2);
        const uint32_t wd = (lo & ~m4) | (hi & m4);
        ins = (wd >> (16u * (j & 1u))) & 0xFFFFu;
        return have;
    };
    bool live = false;
    uint32_t v = SR_RUN;
    auto refill = [&]() {
        /* pf (chunk pfc, issued at an earlier refill) becomes nx once cur reaches pfc - 1;
         * then the chunk after the newest one held or in flight is requested, so two chunks
         * ahead of cur are buffered or on their way */
        if (pfv && !nxv && pfc == tci + 1u) {
            nx = pf;
            nxv = true;
            pfv = false;
        }
        if (pfv && (pfc <= tci || pfc > tci + 2u)) pfv = false;     /* stale: a jump */
        const uint32_t want = nxv ? tci + 2u : tci + 1u;
        if (tn != 0xFFu && !pfv && want * 8u < stride && v == SR_RUN) {   /* not while it waits to hand over */
            pf = ld16(slot_of(tn) + want * 8u);
            pfc = want;
            pfv = true;
        }
    };
    auto on_dump = [&](uint32_t nd) { store_rec(nd, 2u, 0u); };
    auto finish = [&](uint32_t v) {
        if (v == SR_OVF) {               /* to the 256-deep re-run, from scratch */
            const uint32_t pos = gatomic_add((GU32 *)ovf_count, 1u);
            ((GU32 *)ovf_list)[pos] = (uint32_t)sys;
            atomicAdd(&s_cnt[K_OVFRERUN], 1ull);
            return;
        }
        uint32_t ins = 0;
#pragma unroll
        for (uint32_t nd = 0; nd < (uint32_t)NP; ++nd) {   /* unrolled: a fixed store count */
            ins += m.ld(S_CT + nd) >> SC_IP;
            store_rec(nd, ser_final_flags(m, nd), 1u);
        }
        v4u32 res;
        res.x = r.st | (r.dmp << 8); res.y = r.rounds; res.z = r.msgs; res.w = ins;
        ((GV4 *)results)[2 * sys] = res;
        atomicAdd(&s_cnt[K_MSGS], (unsigned long long)r.msgs);
        atomicAdd(&s_cnt[K_INSTRS], (unsigned long long)ins);
        atomicAdd(&s_cnt[K_ROUNDS], (unsigned long long)r.rounds);
        atomicAdd(&s_cnt[K_SYSTEMS], 1ull);
        atomicAdd(&s_cnt[K_STATUS + r.st], 1ull);
        atomicMax(&s_cnt[K_MAXR], (unsigned long long)r.rounds);
    };

    {
        const uint32_t k = claim_next();
        live = k < n;
        if (live) sys = sel(k);
        if (live && serfmt) load_rec(sys);
    }
    v = live ? start() : SR_RUN;
    uint32_t iters = 0, nmac = 0;
#if SIM_TAILPROBE == 2
    /* probe: per lane, the iteration its system started at and whether it was lone at
     * suspension (header word 121), and running maxima / sums published at the kernel's end */
    uint32_t tclaim = 0;
    bool lone0 = live && serfmt && (rr[30].y & 0x100u);
    uint64_t pr_long = 0, pr_last = 0, pr_n4k = 0, pr_nl_it = 0, pr_it = 0, pr_nl_n = 0;
#endif
    /* batched hand-overs: a hand-over is a wave-wide phase (~19k cycles on C3, most of it
     * waits on the claim, the lookup, the successor's rows and the record stores) however
     * few lanes take part, so a finished system waits, its lane idle, until SER_HB lanes of
     * the wave have finished, or the oldest has waited SER_HT iterations, or no running
     * system is left in the wave; then they hand over together (wave-uniform) */
    uint32_t hwait = 0;
    for (;;) {
#pragma unroll 1
        for (int k = 0; k < SER_RF; ++k) {
            /* a lone node's whole transaction at once (ser_macro), else one node-action */
            bool mac = false;
            uint64_t tp0 = 0, tp1 = 0, tp2 = 0;
            if (SER_PROBE >= 2) tp0 = __builtin_amdgcn_s_memtime();
            if (!CAP) {
#pragma unroll
                for (int j = 0; j < SER_MACRO; ++j) {
                    const bool q = live && v == SR_RUN && ser_quiet_lone(r, lim_rsh) && (j == 0 || mac);
                    bool did = false;
                    bool nohave = false;
                    if (SER_PROBE && q) {         /* the instruction not at hand in registers */
                        const uint32_t n0 = dsms::s_ctz(r.A), ip0 = m.ld(S_CT + n0) >> SC_IP, c0 = ip0 >> 3;
                        nohave = !((tn == n0) & ((tci == c0) | ((tci + 1u == c0) & nxv)));
                    }
                    if (SER_PROBE >= 4) {     /* phase cycles of the macro-step (lane 0's view) */
                        uint64_t ts[5] = {0, 0, 0, 0, 0};
                        auto stamp = [&](int i) { __builtin_amdgcn_s_waitcnt(0); ts[i + 1] = __builtin_amdgcn_s_memtime(); };
                        __builtin_amdgcn_s_waitcnt(0);
                        ts[0] = __builtin_amdgcn_s_memtime();
                        if (__ballot(q) && q) did = ser_macro<NP>(m, r, cc, fetch_reg, on_dump, stamp);
                        const uint64_t okb = __ballot(did);
                        if (okb && lane == (uint32_t)__builtin_ctzll(okb)) {
                            atomicAdd(&s_cnt[13], ts[1] - ts[0]);      /* entry + fetch      */
                            atomicAdd(&s_cnt[14], ts[2] - ts[1]);      /* the homes' words   */
                            atomicAdd(&s_cnt[15], ts[3] - ts[2]);      /* decide             */
                            atomicAdd(&s_cnt[16], ts[4] - ts[3]);      /* write-back         */
                        }
                    } else if (__ballot(q) && q) {
                        did = ser_macro<NP>(m, r, cc, fetch_reg, on_dump, [](int) {});
                    }
                    if (SER_PROBE && j == 0) {
                        const uint64_t nh = __ballot(nohave);
                        if (lane == 0) atomicAdd(&s_cnt[8 + 3], 0ull + __builtin_popcountll(nh));
                    }
                    if (SER_PROBE && j == 0) {   /* lane-iterations left to ser_step, by cause */
                        const bool nq_ = live && v == SR_RUN && !q;
                        const uint64_t nq = __ballot(nq_), qn = __ballot(q && !did);
                        const uint64_t mi = __ballot(nq_ && (r.iss & (r.iss - 1u)) != 0u);   /* several may act */
                        if (lane == 0) {
                            atomicAdd(&s_cnt[9], (unsigned long long)__builtin_popcountll(nq));
                            atomicAdd(&s_cnt[10], (unsigned long long)__builtin_popcountll(qn));
                            (void)mi;
                        }
                    }
                    mac = mac || did;
                    nmac += did ? 1u : 0u;
                }
                /* a macro-step that ended the system (the dead-end forward): quiescent */
                if (mac && r.A == 0u) v = SR_DONE;
            }
            if (SER_PROBE) {
                const uint64_t gm = __ballot(live && v == SR_RUN && !mac), mm = __ballot(mac);
                const uint64_t lv = __ballot(live);
                if (lane == 0) {
                    atomicAdd(&s_cnt[8], (unsigned long long)__builtin_popcountll(lv));   /* live lanes */
                    if (__builtin_popcountll(lv) < 32) atomicAdd(&s_cnt[12], 1ull);
                    atomicAdd(&s_cnt[0], 1ull);
                    if (mm) atomicAdd(&s_cnt[1], 1ull);
                    if (gm) atomicAdd(&s_cnt[2], 1ull);
                }
            }
            if (SER_PROBE >= 2) tp1 = __builtin_amdgcn_s_memtime();
            if (live && v == SR_RUN && !mac && (k % SER_GE) == 0) {
                v = ser_step<NP, S_QN, CAP>(m, r, T, fetch, on_dump, lim_rsh, cap);
                ser_cache_clear(cc);
            }
            if (SER_PROBE >= 2) tp2 = __builtin_amdgcn_s_memtime();
            if (SER_PROBE) {
                const uint64_t hm = __ballot(live && v != SR_RUN);
                if (lane == 0 && hm) atomicAdd(&s_cnt[4], 1ull);
            }
            bool hgo = false;
            if (SER_HB > 1) {
                const uint64_t fin = __ballot(live && v != SR_RUN);
                if (fin) {
                    hgo = (uint32_t)__builtin_popcountll(fin) >= (uint32_t)SER_HB ||
                          hwait >= (uint32_t)SER_HT || fin == __ballot(live);
                    hwait = hgo ? 0u : hwait + 1u;
                }
            } else {
                hgo = true;
            }
            if (hgo && live && v != SR_RUN) {
#if SIM_TAILPROBE == 2
                const uint32_t now_it = iters + (uint32_t)k;   /* this iteration (before the claim's k) */
#endif
                uint64_t th0 = 0, th1 = 0, th2 = 0;
                if (SER_PROBE >= 3) th0 = __builtin_amdgcn_s_memtime();
                /* the successor: claimed and looked up first (waits that cover nothing but
                 * older loads, the claim and the lookup), then its record's rows put in
                 * flight before the finished system's record stores: the wait for the rows
                 * (vmcnt counts stores too) is the only one left behind the stores.  Round 5:
                 * C3 42.6 -> 40.4 ms, C5 32.6 -> 30.7 with the claim and the lookup as global,
                 * not flat, accesses (a pending flat operation turns every later wait into a
                 * full one) and the rows before the stores.  Measured slower, not kept:
                 * claiming the successor ahead, at a refill step while the lone node's last
                 * 16-64 instructions run (C5 31.9 ms); records written at their list position
                 * so the claim needs no lookup (C3 +0.3 ms: the budget pass then waits for
                 * the position before the record's stores). */
                wait_vmcnt0();
                const uint32_t k = claim_next();
                const bool nl = k < n;
                const uint32_t ns = nl ? sel(k) : 0u;
                if (nl && serfmt) load_rec(ns);
                if (SER_PROBE >= 3) { __builtin_amdgcn_s_waitcnt(0); th1 = __builtin_amdgcn_s_memtime(); }
#if SIM_TAILPROBE == 2
                {   /* probe: the longest system, and the duration of the system that ends last */
                    const uint64_t dur = (uint64_t)(now_it - tclaim);
                    const uint64_t a = (dur << 32) | (uint64_t)sys;
                    const uint64_t b = ((uint64_t)now_it << 32) | ((uint64_t)lone0 << 31) | dur;
                    pr_long = a > pr_long ? a : pr_long;
                    pr_last = b > pr_last ? b : pr_last;
                    pr_n4k += dur > 4000u ? 1u : 0u;
                    pr_nl_it += lone0 ? 0u : dur;
                    pr_it += dur;
                    pr_nl_n += lone0 ? 0u : 1u;
                    tclaim = now_it;
                    lone0 = nl && serfmt && (rr[30].y & 0x100u);
                }
#endif
                finish(v);
                if (SER_PROBE >= 3) { __builtin_amdgcn_s_waitcnt(0); th2 = __builtin_amdgcn_s_memtime(); }
                live = nl;
                sys = ns;
                v = live ? start() : SR_RUN;
                if (SER_PROBE >= 3) {    /* hand-over cycles: finish, claim, start (lowest lane) */
                    __builtin_amdgcn_s_waitcnt(0);
                    const uint64_t th3 = __builtin_amdgcn_s_memtime();
                    const uint64_t fl = __ballot(true);
                    if (lane == (uint32_t)__builtin_ctzll(fl)) {
                        atomicAdd(&s_cnt[13], th1 - th0);
                        atomicAdd(&s_cnt[14], th2 - th1);
                        atomicAdd(&s_cnt[15], th3 - th2);
                    }
                }
            }
            if (SER_PROBE >= 2 && lane == 0) {   /* cycles: macro phase, one-action phase, hand-over */
                const uint64_t tp3 = __builtin_amdgcn_s_memtime();
                atomicAdd(&s_cnt[5], tp1 - tp0);
                atomicAdd(&s_cnt[6], tp2 - tp1);
                atomicAdd(&s_cnt[7], tp3 - tp2);
            }
        }
        uint64_t tr0 = 0;
        if (SER_PROBE >= 2) tr0 = __builtin_amdgcn_s_memtime();
        refill();
        (void)tr0;
        iters += SER_RF;
        if (__ballot(live) == 0) break;
    }
#if SIM_TAILPROBE == 2
    {
        uint64_t v6[6] = {pr_long, pr_last, pr_n4k, pr_nl_it, pr_it, pr_nl_n};
#pragma unroll
        for (int q = 0; q < 6; ++q) {
            uint64_t x = v6[q];
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t lo = __shfl_xor((uint32_t)x, o, 64), hi = __shfl_xor((uint32_t)(x >> 32), o, 64);
                const uint64_t y = ((uint64_t)hi << 32) | lo;
                x = q < 2 ? (y > x ? y : x) : x + y;
            }
            if (lane == 0) {
                if (q < 2) atomicMax(&Ap->counters[q], (unsigned long long)x);
                else atomicAdd(&Ap->counters[q], (unsigned long long)x);
            }
        }
    }
#endif
    if (lane == 0) {
        atomicAdd(&s_cnt[K_WROUNDS], (unsigned long long)iters);
        atomicAdd(&Ap->counters[K_SERIT], (unsigned long long)iters);
#if SIM_TAILPROBE
        /* probe build: when the serial pass's waves end, ms after the wave started -- slot 34:
         * before 11 ms, 35..38: [10 + k, 11 + k) for k = 1..4, 39: 15 ms and later */
        const uint64_t ms = (__builtin_amdgcn_s_memrealtime() - tprobe0) / 100000u;
        atomicAdd(&Ap->counters[K_SERPROBE + (ms < 11u ? 0u : (ms - 10u < 5u ? ms - 10u : 5u))], 1ull);
#endif
    }
    if (!CAP) {          /* lone-node transaction steps (ser_macro): one atomic per wave */
        uint32_t t = nmac;
        for (int o = 1; o < 64; o <<= 1) t += __shfl_xor(t, o, 64);
        if (lane == 0 && t) atomicAdd(&Ap->counters[K_SERMAC], (unsigned long long)t);
    }
    __syncthreads();
    if (threadIdx.x < K_N) {
        const unsigned long long x = s_cnt[threadIdx.x];
        if (x) {
            if (threadIdx.x == K_MAXR) atomicMax(&Ap->counters[K_MAXR], x);
            else atomicAdd(&Ap->counters[threadIdx.x], x);
        }
    }
}

/* ---- aggregate: the golden-aggregate view of per-system results (dsm_aggregate) --------
 * One lane per system (32-B result: two 16-B loads); per-lane sums, then wave sums by
 * shuffles and one device atomic per slot and workgroup.  The result digest is the sum of
 * per-system fmix64 chains over the absolute system id (dsm_host.c dsm_result_digest). */
constexpr int AGG_SLOTS = 13;      /* systems, msgs, instrs, rounds, max, status x5, dh, fh, digest */
static_assert(AGG_SLOTS <= DSM_NAGG && DSM_AGG_MAX_SLOT == 4, "dsm_aggregate layout");
__global__ void __launch_bounds__(256) agg_kernel(uint64_t n_sys, uint64_t first_sys,
                                                  const uint4 *res, unsigned long long *agg) {
    __shared__ unsigned long long s_a[4][AGG_SLOTS];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    uint64_t v[AGG_SLOTS];
#pragma unroll
    for (int k = 0; k < AGG_SLOTS; ++k) v[k] = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n_sys; i += (uint64_t)gridDim.x * 256) {
        const uint4 a = res[2 * i], b = res[2 * i + 1];
        const uint64_t dh = b.x | ((uint64_t)b.y << 32), fh = b.z | ((uint64_t)b.w << 32);
        const uint32_t st = a.x & 0xFFu;
        v[0] += 1; v[1] += a.z; v[2] += a.w; v[3] += a.y;
        v[4] = a.y > v[4] ? a.y : v[4];
#pragma unroll
        for (uint32_t k = 0; k < 5; ++k) v[5 + k] += st == k ? 1u : 0u;
        v[10] += dh; v[11] += fh;
        uint64_t h = fmix64((first_sys + i) * 0x9E3779B97F4A7C15ULL + 1u);
        h = fmix64(h ^ ((uint64_t)a.x | ((uint64_t)a.y << 32)));
        h = fmix64(h ^ ((uint64_t)a.z | ((uint64_t)a.w << 32)));
        h = fmix64(h ^ dh);
        v[12] += fmix64(h ^ fh);
    }
#pragma unroll
    for (int k = 0; k < AGG_SLOTS; ++k) {
        uint64_t x = v[k];
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t lo = __shfl_xor((uint32_t)x, o, 64), hi = __shfl_xor((uint32_t)(x >> 32), o, 64);
            const uint64_t y = ((uint64_t)hi << 32) | lo;
            x = k == 4 ? (y > x ? y : x) : x + y;
        }
        if (lane == 0) s_a[wv][k] = x;
    }
    __syncthreads();
    if (threadIdx.x < AGG_SLOTS) {
        const uint32_t k = threadIdx.x;
        unsigned long long x = s_a[0][k];
        for (int w = 1; w < 4; ++w) x = k == 4 ? (s_a[w][k] > x ? s_a[w][k] : x) : x + s_a[w][k];
        if (k == 4) atomicMax(&agg[k], x);
        else if (x) atomicAdd(&agg[k], x);
    }
}

/* ---- digest: per-system hashes of the node records ------------------------------------
 * One lane per node record pair; dump_hash sums the 15-word hash of every dumped node's
 * dump record, final_hash the 16-word hash of every final record.  Memory-
 * bound (128 B read per node); keeps the 64-bit hashing out of the transition kernel. */
template <int NP>
__global__ void __launch_bounds__(256) digest_kernel(uint64_t n_sys, const uint4 *recs,
                                                     dsm_sys_result *results,
                                                     unsigned long long *counters) {
    __shared__ unsigned long long s_sum[2][4];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6, node = lane % NP;
    uint64_t adh = 0, afh = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i - node < n_sys * NP;
         i += (uint64_t)gridDim.x * 256) {
        const uint64_t sys = i / NP;
        const bool ok = sys < n_sys;
        uint64_t dh = 0, fh = 0;
        if (ok) {
            const uint4 *r = recs + i * 8;
            const uint32_t dmask = results[sys].status >> 8;
            uint64_t hd = 0x9E3779B97F4A7C15ULL * (uint64_t)(node + 1), hf = hd;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint4 d = r[q], f = r[4 + q];
                const uint32_t dw[4] = {d.x, d.y, d.z, d.w}, fw[4] = {f.x, f.y, f.z, f.w};
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int wi = 4 * q + k;
                    if (wi < 15) hd = fmix64(hd ^ ((uint64_t)dw[k] | ((uint64_t)wi << 32)));
                    hf = fmix64(hf ^ ((uint64_t)fw[k] | ((uint64_t)wi << 32)));
                }
            }
            dh = ((dmask >> node) & 1u) ? hd : 0;
            fh = hf;
        }
        dh = gsum64<NP>(dh);
        fh = gsum64<NP>(fh);
        if (ok && node == 0) {
            results[sys].dump_hash = dh;
            results[sys].final_hash = fh;
            adh += dh;
            afh += fh;
        }
    }
    /* block partial: wave sums, then one write per block */
    for (int o = 1; o < 64; o <<= 1) {
        adh += ((uint64_t)__shfl_xor((uint32_t)(adh >> 32), o, 64) << 32) | __shfl_xor((uint32_t)adh, o, 64);
        afh += ((uint64_t)__shfl_xor((uint32_t)(afh >> 32), o, 64) << 32) | __shfl_xor((uint32_t)afh, o, 64);
    }
    if (lane == 0) { s_sum[0][wv] = adh; s_sum[1][wv] = afh; }
    __syncthreads();
    if (threadIdx.x < 2) {      /* block sums into the counters (sums mod 2^64) */
        const unsigned long long v = s_sum[threadIdx.x][0] + s_sum[threadIdx.x][1] +
                                     s_sum[threadIdx.x][2] + s_sum[threadIdx.x][3];
        if (v) atomicAdd(&counters[threadIdx.x ? K_FHASH : K_DHASH], v);
    }
}

/* ---- trace generator ------------------------------------------------------------------
 * One workgroup iteration = one (system, node) slot of `stride` instructions; each lane
 * produces 16-byte chunks (8 instructions, two splitmix64 calls) and streams them out with
 * non-temporal stores (written once, read later by another kernel). */
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int NP, int DIST, bool FULL>
__global__ void __launch_bounds__(64) gen_kernel(uint64_t seed, int dist_unused, uint64_t first,
                                                  uint64_t n_sys, uint32_t n_instr,
                                                  uint32_t stride, uint16_t *traces,
                                                  uint32_t *counts) {
    const uint32_t cps = stride >> 3;                /* 16-byte chunks per node slot */
    const uint64_t nslots = n_sys * NP;
    const uint64_t gmul = seed * 0x9E3779B97F4A7C15ULL;
    for (uint64_t slot = blockIdx.x; slot < nslots; slot += gridDim.x) {
        const uint64_t sys = slot / NP;
        const uint32_t node = (uint32_t)(slot % NP);
        /* key = (sys << 16) | (node << 12) | (idx >> 2) -- disjoint fields, so + == | */
        const uint64_t base = gmul + ((first + sys) << 16) + ((uint64_t)node << 12);
        u32x4 *dst = reinterpret_cast<u32x4 *>(traces + slot * stride);
        const int dist = DIST;
#pragma unroll 2
        for (uint32_t k = threadIdx.x; k < cps; k += blockDim.x) {
            u32x4 v;
#pragma unroll
            for (int half = 0; half < 2; ++half) {
                const uint32_t i0 = k * 8 + 4 * half;               /* 4 instructions */
                const uint64_t r = splitmix(base + (i0 >> 2));
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const uint32_t ia = i0 + 2 * j;
                    const uint32_t lo = (FULL || ia < n_instr)
                        ? instr_from_bits<NP>((uint32_t)(r >> (32 * j)) & 0xFFFFu, dist) : 0u;
                    const uint32_t hi = (FULL || ia + 1 < n_instr)
                        ? instr_from_bits<NP>((uint32_t)(r >> (32 * j + 16)) & 0xFFFFu, dist) : 0u;
                    v[2 * half + j] = lo | (hi << 16);
                }
            }
            __builtin_nontemporal_store(v, dst + k);
        }
        if (threadIdx.x == 0 && counts) counts[slot] = n_instr;
    }
}

/* ---- kernel table ------------------------------------------------------------------- */
typedef void (*sim_fn)(const SimArgs *);

/* Waves per workgroup of the fast transition kernel.  The micro-op table is one copy per
 * workgroup in LDS; at ring 12 a wave needs ~6 KB of LDS and the kernel fits 5 waves per
 * SIMD (96 VGPRs), so 4-wave groups (5 per CU = 20 waves, 146 KB LDS) fill the CU where
 * 8-wave groups stop at 2 per CU (16 waves; measured 0.6% slower, profiles/README.md). */
constexpr int FW = 4;

template <int NP, bool GEN, int MODE>
sim_fn fast_mode(int ring) {
    /* the inbox depth only moves time, never results: every depth for the bench mode, and
     * the overflow-prone depth 4 (which exercises the 256-deep re-run) for the others */
    switch (ring) {
    case 4: return sim_kernel<NP, 4, FW, GEN, MODE>;
    case 8: if ((MODE & ~(M_NOFF | M_SERB)) == 0) return sim_kernel<NP, 8, FW, GEN, MODE & (M_NOFF | M_SERB)>; break;
    case 16: if ((MODE & ~(M_NOFF | M_SERB)) == 0) return sim_kernel<NP, 16, FW, GEN, MODE & (M_NOFF | M_SERB)>; break;
    default: break;
    }
    return sim_kernel<NP, 12, FW, GEN, MODE>;
}
template <int NP, bool GEN>
sim_fn fast_np_gen(int ring, int mode) {
    switch (mode) {
    case 1: return fast_mode<NP, GEN, 1>(ring);
    case 2: return fast_mode<NP, GEN, 2>(ring);
    case 3: return fast_mode<NP, GEN, 3>(ring);
    case 4: return fast_mode<NP, GEN, 4>(ring);
    case 5: return fast_mode<NP, GEN, 5>(ring);
    case 6: return fast_mode<NP, GEN, 6>(ring);
    case 7: return fast_mode<NP, GEN, 7>(ring);
    case M_LIM: return fast_mode<NP, GEN, M_LIM>(ring);
    case M_NOFF:                        /* packed path only (ffscan_kernel reads traces); the
                                         * fused generator has no plain kernel: mode 0 */
        if constexpr (!GEN) return fast_mode<NP, GEN, M_NOFF>(ring);
        else return fast_mode<NP, GEN, 0>(ring);
    case M_NOFF | M_SERB:
        if constexpr (!GEN) return fast_mode<NP, GEN, M_NOFF | M_SERB>(ring);
        else return fast_mode<NP, GEN, 0>(ring);
    default: return fast_mode<NP, GEN, 0>(ring);
    }
}
sim_fn pick_fast(int np, int ring, bool gen, int mode) {
    if (np == 4) return gen ? fast_np_gen<4, true>(ring, mode) : fast_np_gen<4, false>(ring, mode);
    return gen ? fast_np_gen<8, true>(ring, mode) : fast_np_gen<8, false>(ring, mode);
}
template <int NP, bool GEN>
sim_fn fb_np_gen(int mode) {
    switch (mode & 7) {       /* the re-run always reads the limits (LIM) */
    case 1: return sim_kernel<NP, FB_RING, 1, GEN, 1, 1>;
    case 2: return sim_kernel<NP, FB_RING, 1, GEN, 2, 1>;
    case 3: return sim_kernel<NP, FB_RING, 1, GEN, 3, 1>;
    case 4: return sim_kernel<NP, FB_RING, 1, GEN, 4, 1>;
    case 5: return sim_kernel<NP, FB_RING, 1, GEN, 5, 1>;
    case 6: return sim_kernel<NP, FB_RING, 1, GEN, 6, 1>;
    case 7: return sim_kernel<NP, FB_RING, 1, GEN, 7, 1>;
    default: return sim_kernel<NP, FB_RING, 1, GEN, 0, 1>;
    }
}
sim_fn pick_fallback(int np, bool gen, int mode) {
    if (np == 4) return gen ? fb_np_gen<4, true>(mode) : fb_np_gen<4, false>(mode);
    return gen ? fb_np_gen<8, true>(mode) : fb_np_gen<8, false>(mode);
}
int lds_bytes(int ring, int waves) {
    return waves * (8 * 64 * 4 + 4 * 64 * 4 + ring * 64 * 4 + 128 * 4 + 64 * 4 + K_N * 8) + DT_TABLE_WORDS * 4;
}

/* writes a run's argument blocks (passed by value in the kernarg segment) to device memory,
 * in stream order: no pinned staging buffer, so nothing for the host to wait on */
__global__ void __launch_bounds__(64) args_kernel(SimArgsPack p, SimArgs *dst) {
    constexpr int W = (int)(sizeof(SimArgsPack) / 4);
    const uint32_t *s = reinterpret_cast<const uint32_t *>(&p);
    uint32_t *d = reinterpret_cast<uint32_t *>(dst);
    for (int i = threadIdx.x; i < W; i += 64) d[i] = s[i];
}
static_assert(sizeof(SimArgsPack) % 4 == 0, "SimArgsPack words");

}  // namespace

/* ====================================================================================== */
/* C ABI                                                                                   */
/* ====================================================================================== */


#define CTRL_WORDS 2048
#define CTRL_FAST 0
#define CTRL_FB 256
#define CTRL_OVF 512
#define CTRL_RES 1024       /* claim shards of the resume pass */
#define CTRL_SUSP 1536      /* systems the budget pass suspended (the short class with SER_LONG) */
#define CTRL_SUSPL 1568     /* ... of the long class (SER_LONG), listed from the top down */
#define CTRL_SCAN 1792      /* ffscan_kernel's sample counts */

/* Two-pass schedule (bench mode: MODE 0, packed traces).  A system's length is unknown until
 * it ends, and ~14% of C3 systems run ~12.5k rounds against a median of ~650: in one
 * persistent launch the long systems claimed last set the kernel's end at low occupancy.  The
 * budget pass therefore runs every system for at most 1 << log2 rounds and suspends the rest
 * (their state to HBM); the resume pass continues those (almost all long, of similar
 * remaining length), sizing its own grid from the device-resident count.  Results are
 * identical: a system's rounds run in the same order, only split across two launches.
 * With the serial resume pass (ser_kernel) the budget is 2^10 (C3: 2^10 / 2^12 equal, the
 * tail systems of either budget land 4.5 / 2.3 to a lane; C5: 89.9 vs 101.8 ms), the
 * fast-forward kernel's 2^9; late budget 2^9 (off at a budget <= 2^9).  dsm_set_budget
 * (or DSM_BUDGET_LOG2 / DSM_LATE_LOG2 / DSM_FF_BUDGET_LOG2 in the environment at dsm_open)
 * change them; budget 0 = one pass. */
static uint32_t env_u32(const char *name, uint32_t dflt) {
    const char *e = getenv(name);
    if (!e || !*e) return dflt;
    const long v = strtol(e, nullptr, 10);
    return v < 0 ? 0u : (uint32_t)v;
}

#define ensure dsm_ensure

extern "C" int dsm_device_count(int *count) {
    if (!count) return DSM_E_INVAL;
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
    *count = c;
    return DSM_OK;
}

extern "C" int dsm_open(int device, const dsm_config *cfg, dsm_ctx **out) {
    if (!cfg || !out) return DSM_E_INVAL;
    *out = nullptr;
    if (cfg->np != 4 && cfg->np != 8) return DSM_E_INVAL;
    if (cfg->max_instr == 0 || cfg->max_instr > DSM_MAX_INSTR || (cfg->max_instr & 7u)) return DSM_E_INVAL;
    int ring = cfg->ring_cap ? (int)cfg->ring_cap : 12;
    if (ring != 4 && ring != 8 && ring != 12 && ring != 16) return DSM_E_INVAL;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return DSM_E_DEVICE;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return DSM_E_DEVICE;
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return DSM_E_DEVICE;
    if (hipSetDevice(device) != hipSuccess) return DSM_E_DEVICE;
    dsm_ctx *c = (dsm_ctx *)calloc(1, sizeof(dsm_ctx));
    if (!c) return DSM_E_NOMEM;
    c->device = device;
    c->cfg = *cfg;
    c->sched_thresh = DSM_SCHED_LOCKSTEP;
    c->ring = ring;
    c->cus = prop.multiProcessorCount;
    /* tuning knobs: read here once, reported by dsm_launch_info_get */
    c->budget_log2 = env_u32("DSM_BUDGET_LOG2", 12);
    if (c->budget_log2 >= RSH_MAX) c->budget_log2 = 0;
    /* the fast-forward kernel's budget in rounds (0: the plain budget); DSM_FF_BUDGET_LOG2,
     * if set, gives it as a power of two */
    c->ff_budget_log2 = env_u32("DSM_FF_BUDGET_LOG2", 0);
    if (c->ff_budget_log2 >= RSH_MAX) c->ff_budget_log2 = 0;
    c->ff_budget_rounds = getenv("DSM_FF_BUDGET_LOG2") ? (c->ff_budget_log2 ? 1u << c->ff_budget_log2 : 0u)
                                                       : env_u32("DSM_FF_BUDGET_ROUNDS", 448);
    if (c->ff_budget_rounds >= (1u << RSH_MAX)) c->ff_budget_rounds = 0;
    /* the late budget (a shorter budget once a wave finds no new system) is off: with
     * suspend-on-lone it only cut multi-node systems short into the serial pass, where they
     * take one node-action per step (C3 late 2^9 / 2^10 / 2^11 / off: 50.5 / 47.6 / 45.8 /
     * 42.6 ms) */
    c->late_log2 = env_u32("DSM_LATE_LOG2", 0);
    c->round_limit_log2 = RSH_MAX;
    c->inbox_limit = FB_RING;
    c->ff_mode = DSM_FF_AUTO;
    c->serial = (int)env_u32("DSM_SERIAL", 1);
    /* the budget pass checks for quiet-lone systems every DSM_LONE rounds (0: never), from
     * round DSM_LONE_MIN on (160, round 6: C5 29.4 -> 28.5 ms, C3 within its spread; 128 costs
     * C3 +0.4, 96 and below cost C5 3+ ms: too many multi-node systems reach the serial pass) */
    c->lone_rounds = env_u32("DSM_LONE", 8);
    c->lone_min = env_u32("DSM_LONE_MIN", 160);

    c->fmt_tile = (int)env_u32("DSM_FMT", 132);
    c->parse_bpl = (int)env_u32("DSM_PARSE_BPL", 32);
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc((void **)&c->d_ctrl, CTRL_WORDS * sizeof(unsigned int)) != hipSuccess ||
        hipMalloc((void **)&c->d_args, sizeof(SimArgsPack)) != hipSuccess ||
        hipMalloc((void **)&c->d_cnt, sizeof(dsm_counters)) != hipSuccess ||
        hipMalloc((void **)&c->d_table, DT_TABLE_WORDS * sizeof(uint32_t)) != hipSuccess) {
        dsm_close(c);
        return DSM_E_DEVICE;
    }
    {
        static uint32_t tab[DT_TABLE_WORDS];
        if (dt_build(tab) > DT_ENTRIES || hipMemcpy(c->d_table, tab, sizeof tab, hipMemcpyHostToDevice) != hipSuccess) {
            dsm_close(c);
            return DSM_E_DEVICE;
        }
    }
    if (cfg->flags & DSM_F_TIMING) {
        for (int i = 0; i < DSM_TIMING_RING; ++i)
            if (hipEventCreate(&c->tev0[i]) != hipSuccess || hipEventCreate(&c->tev1[i]) != hipSuccess) {
                dsm_close(c);
                return DSM_E_DEVICE;
            }
    }
    *out = c;
    return DSM_OK;
}

extern "C" void dsm_close(dsm_ctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    void *ptrs[] = {c->d_ctrl, c->d_args, c->d_ovf_list, c->d_susp, c->d_susp_list, c->d_spill,
                    c->d_traces, c->d_counts,
                    c->d_res, c->d_cnt, c->d_recs, c->d_table, c->d_issue, c->d_issue_n};
    for (void *p : ptrs) if (p) (void)hipFree(p);
    dsm_text_release(c);
    for (int i = 0; i < DSM_TIMING_RING; ++i) {
        if (c->tev0[i]) (void)hipEventDestroy(c->tev0[i]);
        if (c->tev1[i]) (void)hipEventDestroy(c->tev1[i]);
    }
    if (c->stream) (void)hipStreamDestroy(c->stream);
    free(c);
}

extern "C" int dsm_launch_info_get(dsm_ctx *c, dsm_launch_info *info) {
    if (!c || !info) return DSM_E_INVAL;
    if (c->last_pair) {
        /* the trace scan chose the pair's kernel on the device: wait for the run, read the
         * verdict (ff_verdict) and report the passes that actually ran (one pass at budget
         * 0: only the kernel it picked) */
        uint32_t scan[2] = {0, 0};
        HIPCK(hipSetDevice(c->device));
        HIPCK(hipStreamSynchronize(c->last_st));
        HIPCK(hipMemcpy(scan, c->d_ctrl + CTRL_SCAN, sizeof scan, hipMemcpyDeviceToHost));
        const bool ff = scan[1] != 0u && (uint64_t)scan[1] * 16u >= scan[0];
        c->info.ff_picked = ff ? 1 : 0;
        if (c->last_blog) {
            c->info.resume_form = ff ? DSM_RESUME_FASTFORWARD
                                     : (c->last_use_ser ? DSM_RESUME_SERIAL : DSM_RESUME_LOCKSTEP);
            c->info.resume_blocks = (ff || !c->last_use_ser) ? c->last_grid_fast : c->last_ser_blocks;
            c->info.budget_rounds = (int)((ff && c->last_thr_ff) ? c->last_thr_ff : 1u << c->last_blog);
            /* the budget pass runs on a plain kernel: with the serial resume, the M_SERB one
             * unless the verdict picked the fast-forward resume (SimArgs::split) */
            c->info.budget_mode = (!ff && c->last_use_ser) ? (M_NOFF | M_SERB) : M_NOFF;
            c->info.resume_mode = ff ? 0 : (c->last_use_ser ? -1 : M_NOFF);
        } else {
            c->info.budget_mode = ff ? 0 : M_NOFF;
            c->info.resume_mode = -1;
        }
        c->last_pair = 0;
    }
    *info = c->info;
    return DSM_OK;
}

/* the non-default compile-time knobs of this build ("" for the default build): A/B and probe
 * variants (tools/build_variant.sh) label their launches apart, and a probe build whose
 * results are not valid for timing (TRAFFIC_PROBE, SIM_TAILPROBE, SER_PROBE) says so */
static const char *build_variant() {
    static char tag[160];
    if (tag[0]) return tag[1] ? tag + 1 : "";
    int n = snprintf(tag, sizeof tag, "#");
    auto add = [&](const char *name, long v, long def) {
        if (v != def && n < (int)sizeof tag) n += snprintf(tag + n, sizeof tag - n, " %s=%ld", name, v);
    };
    add("SIM_BF", SIM_BF, 0);
    add("SER_LONG", SER_LONG, 0);
    add("REC_PROBE", REC_PROBE, 0);
    add("SIM_UNI", SIM_UNI, 1);
    add("SIM_RFL", SIM_RFL, 1);
    add("SIM_R2", SIM_R2, 0);
    add("SIM_TAILPROBE", SIM_TAILPROBE, 0);
    add("TRAFFIC_PROBE", TRAFFIC_PROBE, 0);
    add("SER_PROBE", SER_PROBE, 0);
    add("SER_HB", SER_HB, 8);
    add("SER_HT", SER_HT, 32);
    add("SER_RF_DEF", SER_RF_DEF, 8);
    add("SER_MACRO_DEF", SER_MACRO_DEF, 1);
    add("FF_LONG", FF_LONG, 1);
    add("FF_LONG_U", FF_LONG_U, 8);
    add("SER_DEAD_FWD", SER_DEAD_FWD, 1);
    add("SER_NOTICE_HOME", SER_NOTICE_HOME, 1);
    add("SER_DUMP", SER_DUMP, 0);
    return tag[1] ? tag + 1 : "";
}

extern "C" int dsm_launch_kernel_names(const dsm_launch_info *info, char *buf, size_t cap) {
    if (!info || !buf) return DSM_E_INVAL;
    char b[2][96];
    auto sim = [&](char *o, int m) {
        snprintf(o, 96, "sim_kernel<%d, %d, %d, %s, %d, %d>", info->np, info->ring_cap,
                 info->block_threads / 64, info->gen ? "true" : "false", m, info->occ);
    };
    int n;
    if (info->budget_mode < 0) {
        n = snprintf(buf, cap, "none");
    } else if (info->resume_form == DSM_RESUME_NONE) {
        sim(b[0], info->budget_mode);
        n = snprintf(buf, cap, "run=%s", b[0]);
    } else {
        sim(b[0], info->budget_mode);
        if (info->resume_mode >= 0) sim(b[1], info->resume_mode);
        else snprintf(b[1], 96, "ser_kernel<%d, %s>", info->np, info->ser_cap ? "true" : "false");
        n = snprintf(buf, cap, "budget=%s resume=%s", b[0], b[1]);
    }
    const char *v = build_variant();
    if (n >= 0 && *v && (size_t)n < cap) n += snprintf(buf + n, cap - n, " [variant:%s]", v);
    return (n < 0 || (size_t)n >= cap) ? DSM_E_INVAL : n;
}

extern "C" int dsm_set_budget(dsm_ctx *c, uint32_t budget_log2, uint32_t late_log2) {
    if (!c || budget_log2 >= RSH_MAX || late_log2 >= RSH_MAX) return DSM_E_INVAL;
    c->budget_log2 = budget_log2;
    c->late_log2 = late_log2;
    return DSM_OK;
}

extern "C" int dsm_set_round_limit(dsm_ctx *c, uint32_t limit_log2) {
    if (!c || limit_log2 > RSH_MAX) return DSM_E_INVAL;
    c->round_limit_log2 = limit_log2 ? limit_log2 : RSH_MAX;
    if (c->round_limit_log2 < 1) return DSM_E_INVAL;
    return DSM_OK;
}

extern "C" int dsm_set_fast_forward(dsm_ctx *c, int mode) {
    if (!c || mode < DSM_FF_OFF || mode > DSM_FF_AUTO) return DSM_E_INVAL;
    c->ff_mode = mode;
    return DSM_OK;
}

extern "C" int dsm_set_inbox_limit(dsm_ctx *c, uint32_t cap) {
    if (!c || cap > (uint32_t)FB_RING) return DSM_E_INVAL;
    c->inbox_limit = cap ? cap : (uint32_t)FB_RING;
    return DSM_OK;
}

/* Run the transition kernel (+ resume pass, 256-deep re-run of overflowing systems, digest).
 * Everything is enqueued on `st`; the host never waits. */
static int run_engine(dsm_ctx *c, bool gen, const dsm_gen *g, uint64_t first_sys,
                      const uint16_t *d_traces, const uint32_t *d_counts, uint64_t n_sys,
                      dsm_sys_result *d_results, dsm_counters *d_counters, hipStream_t st) {
    if (n_sys == 0) {    /* nothing launched: the launch info says so */
        c->last_pair = 0;
        c->info.grid_blocks = c->info.block_threads = c->info.resume_blocks = 0;
        c->info.budget_log2 = c->info.late_log2 = c->info.budget_rounds = c->info.ff_picked = 0;
        c->info.budget_mode = c->info.resume_mode = -1;
        c->info.resume_form = DSM_RESUME_NONE;
        return DSM_OK;
    }
    if (n_sys > 0xFFFFFFFFull) return DSM_E_INVAL;
    HIPCK(hipSetDevice(c->device));
    const int np = c->cfg.np, gpw = 64 / np;
    const bool tr = (c->cfg.flags & DSM_F_ISSUE_TRACE) != 0;
    int mode = ((c->cfg.flags & DSM_F_TYPE_COUNTS) ? M_TC : 0) | (tr ? M_TR : 0) |
               (c->sched_thresh < DSM_SCHED_LOCKSTEP ? M_SX : 0);
    /* the bench mode with a round limit or an inbox limit below the fast ring */
    if (mode == 0 && (c->round_limit_log2 != RSH_MAX || c->inbox_limit < (uint32_t)c->ring)) mode = M_LIM;
    /* the bench mode on the packed path: the hit-run fast-forward per dsm_set_fast_forward;
     * in auto, a pair of launches per pass, picked on the device by ffscan_kernel */
    const bool plain_only = mode == 0 && !gen && c->ff_mode == DSM_FF_OFF;
    const bool pair = mode == 0 && !gen && c->ff_mode == DSM_FF_AUTO;
    /* two-pass schedule on the packed path in bench mode */
    const uint32_t blog = ((mode & ~M_LIM) == 0 && !gen) ? c->budget_log2 : 0u;
    /* the resume pass in serial form (ser_kernel) unless fast-forward is forced; with the
     * fast-forward pair, the trace scan's verdict picks between it and the fast-forward
     * lock-step resume */
    const bool use_ser = blog && c->serial && c->ff_mode != DSM_FF_ON;
    /* plain budget kernels: M_SERB (suspend-on-lone, serial-form record) where the serial
     * pass resumes; the pair launches both and the verdict keeps one (SimArgs::split) */
    const int plain_mode = use_ser ? (M_NOFF | M_SERB) : M_NOFF;
    const sim_fn fast = pick_fast(np, c->ring, gen, plain_only ? plain_mode : mode), fb = pick_fallback(np, gen, mode);
    const sim_fn fast_nf = pair ? pick_fast(np, c->ring, gen, M_NOFF) : nullptr;
    const sim_fn fast_serb = pair && use_ser ? pick_fast(np, c->ring, gen, M_NOFF | M_SERB) : nullptr;
    int nb_fast = 0, nb_fb = 0;
    HIPCK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb_fast, (const void *)fast, 64 * FW, 0));
    HIPCK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb_fb, (const void *)fb, 64, 0));
    if (nb_fast < 1 || nb_fb < 1) return DSM_E_DEVICE;
    uint64_t want = (n_sys + (uint64_t)(FW * gpw) - 1) / (uint64_t)(FW * gpw);
    const int grid_max = nb_fast * c->cus;
    int grid_fast = (int)((uint64_t)grid_max < want ? (uint64_t)grid_max : want);
    int grid_fb = nb_fb * c->cus;
    if (grid_fb > 1024) grid_fb = 1024;
    uint64_t dblocks = (n_sys * np + 255) / 256;
    if (dblocks > (uint64_t)c->cus * 8) dblocks = (uint64_t)c->cus * 8;
    int rc;
    if ((rc = ensure(&c->d_ovf_list, &c->ovf_cap, (size_t)n_sys))) return rc;
    const int ring_eff = (mode && c->ring != 4) ? 12 : c->ring;   /* fast_mode's choice */
    if (blog) {
        const size_t sw = (size_t)np * susp_words(ring_eff) > (size_t)ssusp_words(ring_eff)
                              ? (size_t)np * susp_words(ring_eff) : (size_t)ssusp_words(ring_eff);
        if ((rc = ensure(&c->d_susp, &c->susp_cap, (size_t)n_sys * sw))) return rc;
        if ((rc = ensure(&c->d_susp_list, &c->susp_list_cap, (size_t)n_sys))) return rc;
    }
    if ((rc = ensure(&c->d_recs, &c->recs_cap, (size_t)n_sys * np * 8))) return rc;
    /* the serial pass's grid: one workgroup per CU, fewer when the ensemble cannot fill
     * them (at most n_sys systems are suspended); its spill FIFOs: S_SPILL words per lane
     * (96 MiB on 256 CUs, 384 KiB per workgroup) */
    const int ser_blocks = (int)((uint64_t)c->cus < (n_sys + 64 * SER_WAVES - 1) / (64 * SER_WAVES)
                                     ? (uint64_t)c->cus : (n_sys + 64 * SER_WAVES - 1) / (64 * SER_WAVES));
    if (use_ser && (rc = ensure(&c->d_spill, &c->spill_cap, (size_t)ser_blocks * 64 * SER_WAVES * dsms::S_SPILL))) return rc;
    if (!d_results) {   /* the engine needs the per-system header even if the caller does not */
        if ((rc = ensure(&c->d_res, &c->res_cap, (size_t)n_sys + 1))) return rc;
        d_results = c->d_res;
    }
    if (tr) {
        const size_t cap = (size_t)np * c->cfg.max_instr;
        if ((rc = ensure(&c->d_issue, &c->issue_cap_total, (size_t)n_sys * cap))) return rc;
        if ((rc = ensure(&c->d_issue_n, &c->issue_n_cap, (size_t)n_sys))) return rc;
    }
    if (c->cfg.flags & DSM_F_SNAPSHOTS)   /* nodes that never dump read back as zeros */
        HIPCK(hipMemsetAsync(c->d_recs, 0, (size_t)n_sys * np * 128, st));
    c->recs_n = n_sys;
    HIPCK(hipMemsetAsync(c->d_ctrl, 0, CTRL_WORDS * sizeof(unsigned int), st));

    SimArgsPack pk;
    memset(&pk, 0, sizeof pk);
    SimArgs &A = pk.a[0];
    A.traces = d_traces;
    A.counts = d_counts;
    A.stride = c->cfg.max_instr;
    A.n_instr = gen ? g->n_instr : 0;
    A.n_sys = n_sys;
    A.first_sys = first_sys;
    A.seed = gen ? g->seed : 0;
    A.dist = gen ? g->dist : 0;
    A.results = d_results;
    A.recs = c->d_recs;
    A.counters = reinterpret_cast<unsigned long long *>(d_counters);
    A.claim = c->d_ctrl + CTRL_FAST;
    A.ovf_list = c->d_ovf_list;
    A.ovf_count = c->d_ctrl + CTRL_OVF;
    A.table = c->d_table;
    A.sched_seed = c->sched_seed;
    A.sched_thresh = c->sched_thresh;
    A.lim_rsh = c->round_limit_log2;
    A.icap = c->inbox_limit;
    A.rsh = blog ? blog : RSH_MAX;
    /* the fast-forward kernel's own budget (thr_ff rounds).  A short one suspends every
     * system of a hit-run workload at the same round: each pass then holds the systems of a
     * wave in the same phase, so the groups enter and leave fast-forward mode together and
     * the normal round is skipped more often (measured on C4, budget 256 / 320 / 384 / 416 /
     * 512 / 640 / 1024 / 2048 rounds: 50.9 / 48.7 / 48.3 / 48.4 / 49.0 / 50.0 / 53.4 /
     * 57.7 ms; round 4, with the long runs: 320 / 384 / 416 / 448 / 480 / 512 / 640: 34.8 /
     * 32.2 / 31.3 / 31.0 / 30.9 / 31.2 / 33.9 ms).  Bench mode only: with a round or inbox limit (M_LIM) the kernel always has
     * the fast-forward step and takes the plain budget. */
    A.budget = blog ? 1u : 0u;
    A.thr_ff = (mode == 0) ? c->ff_budget_rounds : 0u;
    A.lone = (use_ser && (plain_only || pair)) ? c->lone_rounds : 0u;   /* serial resume only */
    A.lone_min = c->lone_min;

    /* the serial-form record and suspend-on-lone are compiled into the plain budget kernel
     * only (sim_kernel LONE): runs whose budget pass takes it, the pair's plain half or the
     * plain-only bench mode; with limits (M_LIM) the budget pass writes the lock-step form */
    A.serfmt = (use_ser && (plain_only || pair)) ? 1u : 0u;
    A.split = (pair && use_ser) ? 1u : 0u;
    A.late_rsh = (blog && c->late_log2 > 0 && c->late_log2 < blog) ? c->late_log2 : 0u;
    A.susp = c->d_susp;
    A.susp_list = c->d_susp_list;
    A.susp_count = c->d_ctrl + CTRL_SUSP;
    A.susp_long = c->d_ctrl + CTRL_SUSPL;
    A.susp_cap = (uint32_t)n_sys;
    A.susp_ring = (uint32_t)ring_eff;
    A.spill = c->d_spill;
    if (tr) {
        A.issue = c->d_issue;
        A.issue_n = c->d_issue_n;
        A.issue_cap = (uint32_t)((size_t)np * c->cfg.max_instr);
        c->issue_sys = n_sys;
    }
    SimArgs &B = pk.a[1];           /* 256-deep re-run of the overflow list */
    B = A;
    B.d_n = c->d_ctrl + CTRL_OVF;
    B.list = c->d_ovf_list;
    B.claim = c->d_ctrl + CTRL_FB;
    B.ovf_list = nullptr;
    B.ovf_count = nullptr;
    B.rsh = RSH_MAX;
    B.budget = 0;
    SimArgs &C = pk.a[2];           /* resume pass: the suspended list, count on the device */
    C = A;
    C.n_sys = 0;
    C.d_n = c->d_ctrl + CTRL_SUSP;
    C.list = c->d_susp_list;
    C.claim = c->d_ctrl + CTRL_RES;
    C.rsh = RSH_MAX;
    C.budget = 0;
    C.late_rsh = 0;
    C.resume = 1;
    A.scan = C.scan = c->d_ctrl + CTRL_SCAN;
    A.ffsel = C.ffsel = pair ? 1u : 0u;
    hipLaunchKernelGGL(args_kernel, dim3(1), dim3(64), 0, st, pk, c->d_args);
    HIPCK(hipGetLastError());

    const bool timed = (c->cfg.flags & DSM_F_TIMING) != 0;
    const int slot = (int)(c->runs_timed % DSM_TIMING_RING);
    if (timed) HIPCK(hipEventRecord(c->tev0[slot], st));
    if (pair) {
        const uint32_t S = n_sys < SCAN_SYS ? (uint32_t)n_sys : SCAN_SYS;
        const unsigned sb = (unsigned)((S * (uint32_t)np + 255u) / 256u);
        if (np == 4)
            hipLaunchKernelGGL(ffscan_kernel<4>, dim3(sb), dim3(256), 0, st, d_traces, d_counts,
                               (uint32_t)c->cfg.max_instr, n_sys, c->d_ctrl + CTRL_SCAN,
                               reinterpret_cast<unsigned long long *>(d_counters));
        else
            hipLaunchKernelGGL(ffscan_kernel<8>, dim3(sb), dim3(256), 0, st, d_traces, d_counts,
                               (uint32_t)c->cfg.max_instr, n_sys, c->d_ctrl + CTRL_SCAN,
                               reinterpret_cast<unsigned long long *>(d_counters));
        HIPCK(hipGetLastError());
    }
    for (int pass = 0; pass < (blog ? 2 : 1); ++pass) {
        /* resume pass at the budget pass's grid: it sizes itself from the suspended count;
         * in serial form (ser_kernel) one workgroup per CU, one system per lane */
        const SimArgs *a = (const SimArgs *)(c->d_args + 2 * pass);
        const bool ser = pass == 1 && use_ser;
        if (!ser || pair) {
            hipLaunchKernelGGL(fast, dim3(grid_fast), dim3(64 * FW), 0, st, a);
            HIPCK(hipGetLastError());
        }
        if (ser) {
            /* the CAP build keeps per-node inbox counts for an inbox limit below 256 */
            const bool capb = c->inbox_limit < (uint32_t)FB_RING;
            if (!TRAFFIC_PROBE)
                hipLaunchKernelGGL(np == 4 ? (capb ? ser_kernel<4, true> : ser_kernel<4, false>)
                                           : (capb ? ser_kernel<8, true> : ser_kernel<8, false>),
                                   dim3(ser_blocks), dim3(64 * SER_WAVES), 0, st, a);
            HIPCK(hipGetLastError());
        } else if (pair) {
            hipLaunchKernelGGL(fast_nf, dim3(grid_fast), dim3(64 * FW), 0, st, a);
            HIPCK(hipGetLastError());
            if (pass == 0 && fast_serb) {
                hipLaunchKernelGGL(fast_serb, dim3(grid_fast), dim3(64 * FW), 0, st, a);
                HIPCK(hipGetLastError());
            }
        }
    }
    if (timed) {
        HIPCK(hipEventRecord(c->tev1[slot], st));
        c->runs_timed++;
    }

    hipLaunchKernelGGL(fb, dim3(grid_fb), dim3(64), 0, st, (const SimArgs *)(c->d_args + 1));
    HIPCK(hipGetLastError());

    unsigned long long *dcnt = reinterpret_cast<unsigned long long *>(d_counters);
    if (REC_PROBE) {}
    else if (np == 4)
        hipLaunchKernelGGL(digest_kernel<4>, dim3((unsigned)dblocks), dim3(256), 0, st, n_sys,
                           (const uint4 *)c->d_recs, d_results, dcnt);
    else
        hipLaunchKernelGGL(digest_kernel<8>, dim3((unsigned)dblocks), dim3(256), 0, st, n_sys,
                           (const uint4 *)c->d_recs, d_results, dcnt);
    HIPCK(hipGetLastError());

    c->info.grid_blocks = grid_fast;
    c->info.block_threads = 64 * FW;
    c->info.waves_per_cu = nb_fast * FW;
    c->info.cus = c->cus;
    c->info.ring_cap = ring_eff;
    c->info.resume_blocks = blog ? (use_ser ? ser_blocks : grid_fast) : 0;
    c->info.budget_log2 = (int)blog;
    /* without the pair the host knows the passes; with it, dsm_launch_info_get reads the
     * device's verdict */
    const bool ff_kernel = !plain_only && (mode & (M_TR | M_SX)) == 0;   /* step (0) compiled in */
    c->info.ff_picked = ff_kernel ? 1 : 0;
    c->info.resume_form = !blog ? DSM_RESUME_NONE
                        : use_ser ? DSM_RESUME_SERIAL
                        : (ff_kernel ? DSM_RESUME_FASTFORWARD : DSM_RESUME_LOCKSTEP);
    c->info.budget_rounds = blog ? (int)((ff_kernel && A.thr_ff) ? A.thr_ff : 1u << blog) : 0;
    {   /* the MODE of `fast` as instantiated (fast_np_gen: the fused generator has no plain
         * kernel); with the pair, dsm_launch_info_get replaces these with the picked halves */
        const int fm = plain_only ? plain_mode : mode;
        const int fmode = (gen && (fm & M_NOFF)) ? 0 : fm;
        c->info.budget_mode = fmode;
        c->info.resume_mode = (blog && !use_ser) ? fmode : -1;
    }
    c->info.np = np;
    c->info.gen = gen ? 1 : 0;
    c->info.occ = 5;                 /* sim_kernel's default OCC, every fast instantiation */
    c->info.ser_cap = (use_ser && c->inbox_limit < (uint32_t)FB_RING) ? 1 : 0;
    c->last_st = st;
    c->last_pair = pair ? 1 : 0;
    c->last_use_ser = use_ser ? 1 : 0;
    c->last_grid_fast = grid_fast;
    c->last_ser_blocks = ser_blocks;
    c->last_blog = blog;
    c->last_thr_ff = A.thr_ff;
    c->info.lds_bytes_per_block = lds_bytes(ring_eff, FW);
    c->info.late_log2 = (int)A.late_rsh;
    c->info.round_limit_log2 = (int)c->round_limit_log2;
    c->info.fmt_tile = c->fmt_tile;
    c->info.parse_bpl = c->parse_bpl;
    return DSM_OK;
}


static int validate_host_traces(const dsm_ctx *c, const uint16_t *traces, const uint32_t *counts,
                                 uint64_t n_sys) {
    const int np = c->cfg.np;
    const uint32_t stride = c->cfg.max_instr;
    for (uint64_t s = 0; s < n_sys; ++s)
        for (int nd = 0; nd < np; ++nd) {
            const uint32_t cnt = counts[s * np + nd];
            if (cnt > stride) return DSM_E_INVAL;
            const uint16_t *t = traces + (s * np + nd) * (uint64_t)stride;
            for (uint32_t i = 0; i < cnt; ++i)
                if ((uint32_t)((t[i] >> 12) & 7u) >= (uint32_t)np) return DSM_E_RANGE;
        }
    return DSM_OK;
}

extern "C" int dsm_run_packed_device(dsm_ctx *c, const uint16_t *d_traces, const uint32_t *d_counts,
                                     uint64_t n_sys, dsm_sys_result *d_results,
                                     dsm_counters *d_counters, void *stream) {
    if (!c || (n_sys && (!d_traces || !d_counts)) || !d_counters) return DSM_E_INVAL;
    return run_engine(c, false, nullptr, 0, d_traces, d_counts, n_sys, d_results, d_counters,
                      (hipStream_t)stream);
}

extern "C" int dsm_run_generated_device(dsm_ctx *c, const dsm_gen *g, uint64_t first_sys,
                                        uint64_t n_sys, dsm_sys_result *d_results,
                                        dsm_counters *d_counters, void *stream) {
    if (!c || !g || !d_counters) return DSM_E_INVAL;
    if (g->n_instr > DSM_MAX_INSTR || g->dist < 0 || g->dist > 2) return DSM_E_INVAL;
    return run_engine(c, true, g, first_sys, nullptr, nullptr, n_sys, d_results, d_counters,
                      (hipStream_t)stream);
}

static int finish_host(dsm_ctx *c, uint64_t n_sys, dsm_sys_result *per_sys, dsm_counters *out) {
    if (per_sys && n_sys)
        HIPCK(hipMemcpyAsync(per_sys, c->d_res, n_sys * sizeof(dsm_sys_result), hipMemcpyDeviceToHost, c->stream));
    if (out) HIPCK(hipMemcpyAsync(out, c->d_cnt, sizeof(dsm_counters), hipMemcpyDeviceToHost, c->stream));
    HIPCK(hipStreamSynchronize(c->stream));
    return DSM_OK;
}

extern "C" int dsm_run_packed(dsm_ctx *c, const uint16_t *traces, const uint32_t *counts,
                              uint64_t n_sys, dsm_sys_result *per_sys, dsm_counters *out) {
    if (!c || (n_sys && (!traces || !counts))) return DSM_E_INVAL;
    int rc = validate_host_traces(c, traces, counts, n_sys);
    if (rc) return rc;
    HIPCK(hipSetDevice(c->device));
    const size_t slots = (size_t)n_sys * c->cfg.np;
    if ((rc = ensure(&c->d_traces, &c->traces_cap, slots * c->cfg.max_instr + 8))) return rc;
    if ((rc = ensure(&c->d_counts, &c->counts_cap, slots + 1))) return rc;
    if ((rc = ensure(&c->d_res, &c->res_cap, (size_t)n_sys + 1))) return rc;
    if (n_sys) {
        HIPCK(hipMemcpyAsync(c->d_traces, traces, slots * c->cfg.max_instr * sizeof(uint16_t), hipMemcpyHostToDevice, c->stream));
        HIPCK(hipMemcpyAsync(c->d_counts, counts, slots * sizeof(uint32_t), hipMemcpyHostToDevice, c->stream));
    }
    HIPCK(hipMemsetAsync(c->d_cnt, 0, sizeof(dsm_counters), c->stream));
    if ((rc = run_engine(c, false, nullptr, 0, c->d_traces, c->d_counts, n_sys, c->d_res, c->d_cnt, c->stream))) return rc;
    return finish_host(c, n_sys, per_sys, out);
}

extern "C" int dsm_run_generated(dsm_ctx *c, const dsm_gen *g, uint64_t first_sys, uint64_t n_sys,
                                 dsm_sys_result *per_sys, dsm_counters *out) {
    if (!c || !g) return DSM_E_INVAL;
    int rc;
    HIPCK(hipSetDevice(c->device));
    if ((rc = ensure(&c->d_res, &c->res_cap, (size_t)n_sys + 1))) return rc;
    HIPCK(hipMemsetAsync(c->d_cnt, 0, sizeof(dsm_counters), c->stream));
    if ((rc = dsm_run_generated_device(c, g, first_sys, n_sys, c->d_res, c->d_cnt, c->stream))) return rc;
    return finish_host(c, n_sys, per_sys, out);
}

extern "C" int dsm_generate_device(dsm_ctx *c, const dsm_gen *g, uint64_t first_sys, uint64_t n_sys,
                                   uint16_t *d_traces, uint32_t *d_counts, void *stream) {
    if (!c || !g || !d_traces) return DSM_E_INVAL;
    if (g->n_instr > c->cfg.max_instr || g->dist < 0 || g->dist > 2) return DSM_E_INVAL;
    if (n_sys == 0) return DSM_OK;
    HIPCK(hipSetDevice(c->device));
    uint64_t blocks = n_sys * (uint64_t)c->cfg.np;
    const uint64_t cap = (uint64_t)c->cus * 512;   /* many short-lived blocks: measured best (tools/ab_gen.sh) */
    if (blocks > cap) blocks = cap;
    /* the distribution and "every slot full" are compiled in (no per-instruction selects) */
    const bool full = g->n_instr == c->cfg.max_instr;
    const int np = c->cfg.np;
    using gen_fn = void (*)(uint64_t, int, uint64_t, uint64_t, uint32_t, uint32_t, uint16_t *, uint32_t *);
    static const gen_fn tab[2][3][2] = {
        {{gen_kernel<4, 0, false>, gen_kernel<4, 0, true>}, {gen_kernel<4, 1, false>, gen_kernel<4, 1, true>},
         {gen_kernel<4, 2, false>, gen_kernel<4, 2, true>}},
        {{gen_kernel<8, 0, false>, gen_kernel<8, 0, true>}, {gen_kernel<8, 1, false>, gen_kernel<8, 1, true>},
         {gen_kernel<8, 2, false>, gen_kernel<8, 2, true>}}};
    hipLaunchKernelGGL(tab[np == 8][g->dist][full], dim3((unsigned)blocks), dim3(64), 0, (hipStream_t)stream,
                       g->seed, g->dist, first_sys, n_sys, g->n_instr, c->cfg.max_instr, d_traces, d_counts);
    HIPCK(hipGetLastError());
    return DSM_OK;
}

extern "C" int dsm_aggregate_device(dsm_ctx *c, const dsm_sys_result *d_results, uint64_t n_sys,
                                    uint64_t first_sys, dsm_aggregate *d_agg, void *stream) {
    if (!c || !d_agg || (n_sys && !d_results)) return DSM_E_INVAL;
    if (n_sys == 0) return DSM_OK;
    HIPCK(hipSetDevice(c->device));
    uint64_t blocks = (n_sys + 255) / 256;
    const uint64_t cap = (uint64_t)c->cus * 8;
    if (blocks > cap) blocks = cap;
    hipLaunchKernelGGL(agg_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, n_sys, first_sys,
                       reinterpret_cast<const uint4 *>(d_results), reinterpret_cast<unsigned long long *>(d_agg));
    HIPCK(hipGetLastError());
    return DSM_OK;
}

extern "C" int dsm_kernel_ms_history(dsm_ctx *c, float *ms, uint32_t cap, uint32_t *n) {
    if (!c || !n || (cap && !ms)) return DSM_E_INVAL;
    if (!(c->cfg.flags & DSM_F_TIMING)) return DSM_E_STATE;
    HIPCK(hipSetDevice(c->device));
    uint64_t k = c->runs_timed < DSM_TIMING_RING ? c->runs_timed : DSM_TIMING_RING;
    if (k > cap) k = cap;
    for (uint64_t i = 0; i < k; ++i) {       /* oldest first */
        const int slot = (int)((c->runs_timed - k + i) % DSM_TIMING_RING);
        HIPCK(hipEventSynchronize(c->tev1[slot]));
        HIPCK(hipEventElapsedTime(&ms[i], c->tev0[slot], c->tev1[slot]));
    }
    *n = (uint32_t)k;
    return DSM_OK;
}

extern "C" int dsm_last_kernel_ms(dsm_ctx *c, float *ms) {
    if (!c || !ms) return DSM_E_INVAL;
    if (!(c->cfg.flags & DSM_F_TIMING) || c->runs_timed == 0) return DSM_E_STATE;
    uint32_t n = 0;
    return dsm_kernel_ms_history(c, ms, 1, &n);
}

extern "C" int dsm_get_node_state(dsm_ctx *c, uint64_t sys, int node, dsm_node_state *dump,
                                  dsm_node_state *final_state) {
    if (!c || node < 0 || node >= c->cfg.np) return DSM_E_INVAL;
    if (!(c->cfg.flags & DSM_F_SNAPSHOTS) || !c->d_recs) return DSM_E_STATE;
    if (sys >= c->recs_n) return DSM_E_INVAL;
    HIPCK(hipSetDevice(c->device));
    HIPCK(hipStreamSynchronize(c->stream));
    HIPCK(hipDeviceSynchronize());
    const size_t i = ((size_t)sys * c->cfg.np + node) * 8;
    if (dump) HIPCK(hipMemcpy(dump, c->d_recs + i, sizeof *dump, hipMemcpyDeviceToHost));
    if (final_state) HIPCK(hipMemcpy(final_state, c->d_recs + i + 4, sizeof *final_state, hipMemcpyDeviceToHost));
    return DSM_OK;
}

extern "C" int dsm_set_schedule(dsm_ctx *c, uint64_t seed, uint32_t act_thresh) {
    if (!c) return DSM_E_INVAL;
    c->sched_seed = seed;
    c->sched_thresh = act_thresh >= DSM_SCHED_LOCKSTEP ? DSM_SCHED_LOCKSTEP : act_thresh;
    return DSM_OK;
}

extern "C" int dsm_get_issue_trace(dsm_ctx *c, uint64_t sys, uint32_t *events, uint32_t cap,
                                   uint32_t *n) {
    if (!c || !n || (cap && !events)) return DSM_E_INVAL;
    if (!(c->cfg.flags & DSM_F_ISSUE_TRACE) || !c->d_issue) return DSM_E_STATE;
    if (sys >= c->issue_sys) return DSM_E_INVAL;
    HIPCK(hipSetDevice(c->device));
    HIPCK(hipStreamSynchronize(c->stream));
    HIPCK(hipDeviceSynchronize());
    uint32_t k = 0;
    HIPCK(hipMemcpy(&k, c->d_issue_n + sys, sizeof k, hipMemcpyDeviceToHost));
    const uint32_t per = (uint32_t)(c->cfg.np * c->cfg.max_instr);
    const uint32_t m = k < cap ? k : cap;
    if (m) HIPCK(hipMemcpy(events, c->d_issue + sys * per, m * sizeof(uint32_t), hipMemcpyDeviceToHost));
    *n = k;
    return DSM_OK;
}
