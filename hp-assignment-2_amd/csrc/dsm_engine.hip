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
 *   - node state lives in VGPRs, bit-packed: memory 4 dwords, directory bitVectors 4 dwords,
 *     directory states 2 bits x 16, cache address / value bytes, cache states 2 bits x 4;
 *   - inboxes are LDS rings s_ring[wave][slot][lane] (each lane touches only its own column:
 *     bank = lane % 32, conflict-free);
 *   - one round = every lane takes one action; sends go to a per-lane LDS outbox of two words
 *     (body + destination bitmask; the REPLY_ID INV fan-out is one word with a multi-bit mask),
 *     then each receiver lane appends the words addressed to it in ascending sender order,
 *     which is exactly the reference's (sender, program order) delivery order;
 *   - termination per system by wave ballot; finished systems are replaced from a sharded
 *     device work counter (persistent kernel), so lanes never idle on a long-tail system;
 *   - traces are read as 16-byte chunks per lane (cur + prefetched next) from HBM.
 */
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "dsm.h"

#define DEVI __device__ __forceinline__

namespace {

/* transactionType (assignment.c:20-34) plus the local actions of one round */
enum : uint32_t {
    T_RREQ = 0, T_WREQ = 1, T_RRD = 2, T_RWR = 3, T_RID = 4, T_INV = 5, T_UPG = 6,
    T_WBINV = 7, T_WBINT = 8, T_FLUSH = 9, T_FLINV = 10, T_EVS = 11, T_EVM = 12,
    OP_RD = 13, OP_WR = 14, OP_DUMP = 15, OP_IDLE = 16
};
enum : uint32_t { CM = 0, CE = 1, CS = 2, CI = 3 };   /* cacheLineState :17 */
enum : uint32_t { DEM = 0, DS = 1, DU = 2 };          /* directoryEntryState :18 */

/* ctl word: bits 0-7 pendingWriteValue, then flags */
constexpr uint32_t C_WAIT = 1u << 8, C_DUMPED = 1u << 9, C_OVF = 1u << 10, C_ASSERT = 1u << 11;

/* counter slots (dsm_counters order) */
enum { K_MSGS = 13, K_INSTRS = 14, K_ROUNDS = 15, K_SYSTEMS = 16, K_STATUS = 17, K_DHASH = 22,
       K_FHASH = 23, K_MAXR = 24, K_OVFRERUN = 25, K_N = 32 };

constexpr uint64_t NO_SYS = ~0ull;

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
    int snap;
    dsm_sys_result *results;
    dsm_node_state *snap_dump;
    dsm_node_state *snap_final;
    unsigned long long *partials;   /* [waves][K_N], written once per wave at exit         */
    unsigned int *claim;            /* 8 shard counters, 32 words apart                     */
    uint32_t *ovf_list;             /* fast kernel: overflowing systems for the 256 re-run   */
    unsigned int *ovf_count;
};

/* ---- small bit-field helpers ------------------------------------------------------- */
/* Runtime selection among 4 register words.  Written as masks on purpose: a ?: chain over
 * array elements gets folded into a runtime-indexed load, which sends the array to scratch. */
DEVI uint32_t msk(bool b) { return 0u - (uint32_t)b; }
DEVI uint32_t sel4(const uint32_t (&w)[4], uint32_t q) {
    return (w[0] & msk(q == 0)) | (w[1] & msk(q == 1)) | (w[2] & msk(q == 2)) | (w[3] & msk(q == 3));
}
DEVI uint32_t getb16(const uint32_t (&w)[4], uint32_t i) {
    return __builtin_amdgcn_ubfe(sel4(w, i >> 2), (i & 3) * 8, 8);
}
DEVI void setb16(uint32_t (&w)[4], uint32_t i, uint32_t v) {
    const uint32_t sh = (i & 3) * 8, q = i >> 2, m = 0xFFu << sh, x = v << sh;
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
        const uint32_t sel = msk(q == k) & m;
        w[k] = (w[k] & ~sel) | (x & sel);
    }
}
DEVI uint32_t get8(uint32_t w, uint32_t i) { return __builtin_amdgcn_ubfe(w, i * 8, 8); }
DEVI uint32_t set8(uint32_t w, uint32_t i, uint32_t v) {
    const uint32_t sh = i * 8;
    return (w & ~(0xFFu << sh)) | (v << sh);
}
DEVI uint32_t get2(uint32_t w, uint32_t i) { return __builtin_amdgcn_ubfe(w, i * 2, 2); }
DEVI uint32_t set2(uint32_t w, uint32_t i, uint32_t v) {
    const uint32_t sh = i * 2;
    return (w & ~(3u << sh)) | (v << sh);
}

/* message body: type[0:3] addr[4:10] payload[11:18] r2[19:21] excl[22];
 * ring entry = body | sender << 23; outbox entry = body | destination mask << 24 */
DEVI uint32_t mbody(uint32_t type, uint32_t addr, uint32_t payload = 0, uint32_t r2 = 0,
                    uint32_t excl = 0) {
    return type | (addr << 4) | (payload << 11) | (r2 << 19) | (excl << 22);
}
DEVI uint32_t to(uint32_t body, uint32_t dest) { return body | (1u << (24 + dest)); }

/* ---- hashing / generator (same definitions as DESIGN.md; pinned by tests) ----------- */
DEVI uint64_t fmix64(uint64_t z) {
    z ^= z >> 33; z *= 0xff51afd7ed558ccdULL;
    z ^= z >> 33; z *= 0xc4ceb9fe1a85ec53ULL;
    z ^= z >> 33;
    return z;
}
DEVI uint64_t splitmix(uint64_t z) {
    z += 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
/* One splitmix64 output feeds 4 consecutive instructions, 16 bits each. */
template <int NP>
DEVI uint32_t instr_from_bits(uint32_t h, int dist) {
    const uint32_t wr = h & 1u;
    const uint32_t val = wr ? (h >> 1) & 0xFFu : 0u;
    const uint32_t sel = h >> 9;
    uint32_t addr;
    if (dist == DSM_DIST_HOT) addr = (sel & 3u) * 0x11u;
    else if (dist == DSM_DIST_EVICT) addr = (sel & (uint32_t)(NP * 4 - 1)) * 4u;
    else addr = sel & (uint32_t)(NP * 16 - 1);
    return (wr << 15) | (addr << 8) | val;
}
template <int NP>
DEVI uint32_t gen_instr(uint64_t seed, int dist, uint64_t sys, uint32_t node, uint32_t idx) {
    const uint64_t key = (sys << 16) | ((uint64_t)node << 12) | (uint64_t)((idx & 0xFFFu) >> 2);
    const uint64_t r = splitmix(seed * 0x9E3779B97F4A7C15ULL + key);
    return instr_from_bits<NP>((uint32_t)(r >> (16 * (idx & 3u))) & 0xFFFFu, dist);
}

struct Node {
    uint32_t mem[4], bv[4];
    uint32_t dst;     /* directory states, 2 bits per block                                 */
    uint32_t caddr;   /* cache addresses, one byte per line                                 */
    uint32_t cval;    /* cache values                                                       */
    uint32_t cst;     /* cache states, 2 bits per line                                      */
    uint32_t ctl;     /* pending | C_* flags                                                */
    uint32_t ip;      /* instructions issued                                                */
    uint32_t nins;    /* instructions in this node's trace                                  */
    uint32_t rh;      /* inbox head (bits 0-7) | count << 8                                 */
    uint32_t tc[7];   /* messages handled by type, 16-bit fields (type t: tc[t/2], t%2)      */
    uint64_t dh;      /* hash of the dump snapshot                                          */
};

/* canonical 64-byte record (dsm_node_state) word i (i is a compile-time constant after
 * unrolling, so the switch folds away and no 16-register record is ever live) */
DEVI uint32_t rec_word(const Node &nd, uint32_t flags, int i) {
    switch (i) {
    case 0: case 1: case 2: case 3: return nd.mem[i];
    case 4: case 5: case 6: case 7: return nd.bv[i - 4];
    case 8: case 9: case 10: case 11: {
        const uint32_t e = nd.dst >> (8 * (i - 8));
        return (e & 3u) | (((e >> 2) & 3u) << 8) | (((e >> 4) & 3u) << 16) | (((e >> 6) & 3u) << 24);
    }
    case 12: return nd.caddr;
    case 13: return nd.cval;
    case 14:
        return (nd.cst & 3u) | (((nd.cst >> 2) & 3u) << 8) | (((nd.cst >> 4) & 3u) << 16) |
               (((nd.cst >> 6) & 3u) << 24);
    default: return (nd.ctl & 0xFFu) | (flags << 8) | (nd.ip << 16);
    }
}
template <int NW>
DEVI uint64_t node_hash(uint32_t node, const Node &nd, uint32_t flags) {
    uint64_t h = 0x9E3779B97F4A7C15ULL * (uint64_t)(node + 1);
#pragma unroll
    for (int i = 0; i < NW; ++i) h = fmix64(h ^ ((uint64_t)rec_word(nd, flags, i) | ((uint64_t)i << 32)));
    return h;
}
DEVI void store_rec(dsm_node_state *dst, const Node &nd, uint32_t flags) {
    uint4 *p = reinterpret_cast<uint4 *>(dst);
#pragma unroll
    for (int k = 0; k < 4; ++k)
        p[k] = make_uint4(rec_word(nd, flags, 4 * k), rec_word(nd, flags, 4 * k + 1),
                          rec_word(nd, flags, 4 * k + 2), rec_word(nd, flags, 4 * k + 3));
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
DEVI uint4 ld16(const uint16_t *p) { return *reinterpret_cast<const uint4 *>(p); }

template <int NP, bool GEN>
DEVI void start_system(Node &nd, uint32_t (&cur)[4], uint32_t (&nxt)[4], const uint16_t *&tb,
                       uint64_t sys, uint32_t node, const SimArgs &A) {
    /* initializeProcessor :778-790 and main :142-146 */
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
        const uint32_t b = 20u * node + 4u * k;
        nd.mem[k] = (b & 0xFFu) | (((b + 1) & 0xFFu) << 8) | (((b + 2) & 0xFFu) << 16) |
                    (((b + 3) & 0xFFu) << 24);
        nd.bv[k] = 0;
    }
    nd.dst = 0xAAAAAAAAu;   /* all U */
    nd.caddr = 0xFFFFFFFFu; /* address 0xFF */
    nd.cval = 0;
    nd.cst = 0xFFu;         /* all INVALID */
    nd.ctl = 0;
    nd.ip = 0;
    nd.rh = 0;
#pragma unroll
    for (int k = 0; k < 7; ++k) nd.tc[k] = 0;
    nd.dh = 0;
    if (GEN) {
        nd.nins = A.n_instr;
    } else {
        const uint32_t c = A.counts[sys * NP + node];
        nd.nins = c < A.stride ? c : A.stride;
        tb = A.traces + (sys * NP + node) * (uint64_t)A.stride;
        if (nd.nins > 0) {
            const uint4 v = ld16(tb);
            cur[0] = v.x; cur[1] = v.y; cur[2] = v.z; cur[3] = v.w;
        }
        if (nd.nins > 8) {
            const uint4 v = ld16(tb + 8);
            nxt[0] = v.x; nxt[1] = v.y; nxt[2] = v.z; nxt[3] = v.w;
        }
    }
}

/* ---- the transition kernel ------------------------------------------------------------ *
 * One loop iteration = one lock-step round of every system resident in the wave.  The
 * 13 message handlers + 2 issue paths are evaluated as ONE predicated data flow (a shared
 * decode, per-type predicates, selects): a divergent 17-way switch costs every wave the sum
 * of the taken cases plus their exec-mask bookkeeping, this costs one straight line.  Only
 * the once-per-node dump and the trace-chunk refill are real branches.                    */
template <int NP, int RING, int WAVES, bool GEN>
__global__ void __launch_bounds__(64 * WAVES) sim_kernel(SimArgs A) {
    constexpr int GPW = 64 / NP;
    constexpr uint32_t NPM = (1u << NP) - 1u;

    __shared__ uint32_t s_ring[WAVES][RING][64];                     /* inbox rings      */
    __shared__ __attribute__((aligned(16))) uint32_t s_out[WAVES][128]; /* 2 words / lane */
    __shared__ unsigned long long s_cnt[WAVES][K_N];

    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint32_t node = lane % NP, gbase = lane - node;
    if (lane < K_N) s_cnt[wv][lane] = 0;

    const uint64_t n = A.d_n ? (uint64_t)*A.d_n : A.n_sys;
    const uint64_t pool = (uint64_t)gridDim.x * WAVES * GPW;
    const uint64_t rs = n > pool ? (n - pool + 7) / 8 : 0;
    uint32_t shard = blockIdx.x & 7u, tried = 0;
    const uint64_t G = ((uint64_t)blockIdx.x * WAVES + wv) * GPW + lane / NP;

    Node nd;
    uint32_t cur[4] = {0, 0, 0, 0}, nxt[4] = {0, 0, 0, 0};
    const uint16_t *tb = nullptr;
    uint64_t sys = 0;
    uint32_t rounds = 0, rmsg = 0;
    bool live = false;
    nd.ctl = 0; nd.ip = 0; nd.nins = 0; nd.rh = 0; nd.dh = 0;
#pragma unroll
    for (int k = 0; k < 7; ++k) nd.tc[k] = 0;

    if (G < n) {
        sys = A.list ? (uint64_t)A.list[G] : G;
        live = true;
        start_system<NP, GEN>(nd, cur, nxt, tb, sys, node, A);
    }

    for (;;) {
        if (__ballot(live) == 0) break;

        /* ---- (1) this round's action, from state at the start of the round ---------- */
        const uint32_t cnt0 = nd.rh >> 8, head0 = nd.rh & 0xFFu;
        const bool hasMsg = live && cnt0 != 0;                            /* :158-169 */
        const bool canIssue = live && !hasMsg && !(nd.ctl & C_WAIT);      /* :578-581 */
        const bool doIssue = canIssue && nd.ip < nd.nins;                 /* :590-592 */
        const bool doDump = canIssue && !doIssue && !(nd.ctl & C_DUMPED); /* :688-697 */
        nd.rh = hasMsg ? (((head0 + 1) & (RING - 1)) | ((cnt0 - 1) << 8)) : nd.rh;
        uint32_t w = rmsg, op = rmsg & 15u;
        if (doIssue) {
            uint32_t ins;
            if (GEN) {
                ins = gen_instr<NP>(A.seed, A.dist, A.first_sys + sys, node, nd.ip);
            } else {
                const uint32_t k = nd.ip & 7u, d = sel4(cur, k >> 1);
                ins = (k & 1u) ? (d >> 16) : (d & 0xFFFFu);
            }
            op = (ins >> 15) ? OP_WR : OP_RD;
            w = op | (((ins >> 8) & 0x7Fu) << 4) | ((ins & 0xFFu) << 11);
            nd.ip++;
            if (!GEN && (nd.ip & 7u) == 0 && nd.ip < nd.nins) {           /* next chunk */
#pragma unroll
                for (int k = 0; k < 4; ++k) cur[k] = nxt[k];
                if (nd.ip + 8 < nd.nins) {
                    const uint4 v = ld16(tb + nd.ip + 8);
                    nxt[0] = v.x; nxt[1] = v.y; nxt[2] = v.z; nxt[3] = v.w;
                }
            }
        }
        op = hasMsg ? op : doIssue ? op : doDump ? OP_DUMP : OP_IDLE;

        /* ---- (2) decode + the line / directory entry / memory byte it touches -------- */
        const uint32_t a = (w >> 4) & 0x7Fu, v = (w >> 11) & 0xFFu, r2 = (w >> 19) & 7u;
        const uint32_t excl = (w >> 22) & 1u, s = (w >> 23) & 7u;
        const uint32_t H = a >> 4, blk = a & 15u, idx = a & 3u;          /* :177-184 */
        const uint32_t La = get8(nd.caddr, idx), Lv = get8(nd.cval, idx), Ls = get2(nd.cst, idx);
        const uint32_t Db = getb16(nd.bv, blk), Ds = get2(nd.dst, blk), Mv = getb16(nd.mem, blk);
        const uint32_t pend = nd.ctl & 0xFFu;

        const bool tRREQ = op == T_RREQ, tWREQ = op == T_WREQ, tRRD = op == T_RRD;
        const bool tRWR = op == T_RWR, tRID = op == T_RID, tINV = op == T_INV;
        const bool tUPG = op == T_UPG, tWBINV = op == T_WBINV, tWBINT = op == T_WBINT;
        const bool tFLUSH = op == T_FLUSH, tFLINV = op == T_FLINV, tEVS = op == T_EVS;
        const bool tEVM = op == T_EVM, tRD = op == OP_RD, tWR = op == OP_WR;

        const bool home = (H == node), atR2 = (node == r2);
        const bool hit = (La == a), valid = (Ls != CI), hitv = hit && valid;
        const bool mOrE = (Ls <= CE);
        const uint32_t sbit = 1u << s;
        const bool sSet = (Db & sbit) != 0u;
        const uint32_t ob = Db & NPM;
        const uint32_t own = __builtin_ctz(ob | 0x80000000u);            /* findOwner :98 */
        const bool fwd = (Ds == DEM) && (own != s);      /* owner elsewhere: forward */

        /* reference asserts (:189-190,:213,:299-300,:376-377,:408,:443,:489,:542-543) */
        const bool lineOK = hit || La == 0xFFu || !valid;
        const bool emNoOwner = (Ds == DEM) && ob == 0u;
        const bool issueBad = (tRD || tWR) && H >= (uint32_t)NP;
        const bool asrt = ((tRREQ || tWREQ || tUPG || tEVM) && !home) ||
                          ((tRREQ || tWREQ) && emNoOwner) || (tRWR && !lineOK) ||
                          (tFLINV && atR2 && !lineOK) || issueBad;
        const bool rreq = tRREQ && home && !emNoOwner;
        const bool wreq = tWREQ && home && !emNoOwner;
        const bool upg = tUPG && home;

        /* memory: WRITE_REQUEST :379, FLUSH :276, FLUSH_INVACK :478, EVICT_MODIFIED :544 */
        const uint32_t nMv = (home && (tWREQ || tFLUSH || tFLINV || tEVM)) ? v : Mv;

        /* directory */
        const uint32_t evDb = Db & ~sbit;
        const uint32_t rem = __builtin_popcount(evDb & NPM);
        const bool evsH = tEVS && home && sSet;                           /* :501-521 */
        uint32_t nDb = Db, nDs = Ds;
        nDb = rreq ? ((Ds == DU) ? sbit : (Db | sbit)) : nDb;            /* :196-234 */
        nDs = rreq ? (((Ds == DU) || (Ds == DEM && !fwd)) ? DEM : DS) : nDs;
        nDb = (wreq || upg) ? sbit : nDb;                                /* :381-433, :302-327 */
        nDs = (wreq || upg) ? DEM : nDs;
        nDb = (tFLINV && home) ? (1u << r2) : nDb;                       /* :479-480 */
        nDs = (tFLINV && home) ? DEM : nDs;
        nDb = evsH ? evDb : nDb;
        nDs = evsH ? ((rem == 0) ? DU : (rem == 1 && Ds == DS) ? DEM : Ds) : nDs;
        const bool evmClr = tEVM && home && Ds == DEM && sSet;            /* :545-547 */
        nDb = evmClr ? 0u : nDb;
        nDs = evmClr ? DU : nDs;

        /* sends: o0 = victim / reply / forward / flush / INV fan-out, o1 = request */
        uint32_t o0 = 0;
        o0 = rreq ? (fwd ? to(mbody(T_WBINT, a, 0, s), own)
                         : to(mbody(T_RRD, a, Mv, 0, Ds != DS ? 1u : 0u), s)) : o0;
        o0 = wreq ? (fwd ? to(mbody(T_WBINV, a, 0, s), own)
                         : (Ds == DS) ? to(mbody(T_RID, a, Db & ~sbit & 0xFFu), s)
                                      : to(mbody(T_RWR, a), s)) : o0;
        o0 = upg ? to(mbody(T_RID, a, (Ds == DS) ? (Db & ~sbit & 0xFFu) : 0u), s) : o0;
        o0 = (evsH && rem == 1 && Ds == DS)
                 ? to(mbody(T_EVS, a), __builtin_ctz((evDb & NPM) | 0x80000000u)) : o0;
        const bool flushOut = (tWBINT || tWBINV) && hit && mOrE;          /* :251-264, :453-466 */
        o0 = flushOut ? (mbody(tWBINT ? T_FLUSH : T_FLINV, a, Lv, r2) | (1u << (24 + H)) |
                         (1u << (24 + r2))) : o0;
        const uint32_t invm = v & NPM & ~(1u << node);                   /* :350-362 */
        o0 = (tRID && hit && invm) ? (mbody(T_INV, a) | (invm << 24)) : o0;
        const bool isIssue = (tRD || tWR) && !issueBad;
        const bool installRd = tRRD || (tFLUSH && atR2);                 /* :238-247, :286-295 */
        const bool evict = (La != 0xFFu) && valid &&                      /* :742-773 */
                           ((installRd && !hit) || (isIssue && !hitv));
        o0 = evict ? to((Ls == CM) ? mbody(T_EVM, La, Lv) : mbody(T_EVS, La), La >> 4) : o0;
        const bool sendReq = isIssue && (!hitv || (tWR && Ls == CS));     /* :612-629, :646-684 */
        const uint32_t o1 = sendReq ? to(mbody(tRD ? T_RREQ : (hitv ? T_UPG : T_WREQ), a,
                                                (tWR && !hitv) ? v : 0u), H) : 0u;

        /* cache line */
        const bool installWr = (tRWR || (tFLINV && atR2)) && lineOK;      /* :437-449, :483-495 */
        const bool issueMiss = isIssue && !hitv;
        const bool wrHit = tWR && !issueBad && hitv;                      /* :640-659 */
        const bool ridUp = tRID && hit && Ls != CM;                       /* :332-336 */
        const uint32_t nLa = (installRd || installWr || issueMiss) ? a : La;
        uint32_t nLv = Lv;
        nLv = ridUp ? pend : nLv;
        nLv = wrHit ? v : nLv;
        nLv = issueMiss ? 0u : nLv;
        nLv = installWr ? (tRWR ? pend : v) : nLv;
        nLv = installRd ? v : nLv;
        uint32_t nLs = Ls;
        nLs = (tEVS && !home && s == H && hit && Ls == CS) ? CE : nLs;    /* :526-532 */
        nLs = (tINV && hit && (Ls == CS || Ls == CE)) ? CI : nLs;         /* :366-373 */
        nLs = flushOut ? (tWBINT ? CS : CI) : nLs;
        nLs = ridUp ? CM : nLs;
        nLs = wrHit ? CM : nLs;
        nLs = issueMiss ? CI : nLs;
        nLs = installWr ? CM : nLs;
        nLs = installRd ? ((tRRD && excl) ? CE : CS) : nLs;

        /* waitingForReply / pendingWriteValue / assert flag */
        const bool clrWait = installRd || installWr || tRID;
        uint32_t ctl = nd.ctl;
        ctl = sendReq ? (ctl | C_WAIT) : clrWait ? (ctl & ~C_WAIT) : ctl;
        ctl = (tWR && !issueBad) ? ((ctl & ~0xFFu) | v) : ctl;           /* :633 */
        ctl = asrt ? (ctl | C_ASSERT) : ctl;
        nd.ctl = ctl;

        /* ---- (3) write back (idle lanes rewrite unchanged values) ------------------- */
        nd.caddr = set8(nd.caddr, idx, nLa);
        nd.cval = set8(nd.cval, idx, nLv);
        nd.cst = set2(nd.cst, idx, nLs);
        nd.dst = set2(nd.dst, blk, nDs);
        setb16(nd.bv, blk, nDb);
        setb16(nd.mem, blk, nMv);
        {
            const uint32_t inc = (op <= T_EVM) ? (1u << ((op & 1u) * 16)) : 0u, q = op >> 1;
#pragma unroll
            for (uint32_t k = 0; k < 7; ++k) nd.tc[k] += (q == k) ? inc : 0u;
        }
        if (doDump) {                                                    /* :688-697 */
            nd.ctl |= C_DUMPED;
            nd.dh = node_hash<15>(node, nd, 2u);
            if (A.snap) store_rec(&A.snap_dump[sys * NP + node], nd, 2u);
        }

        /* ---- (4) end-of-round delivery: ascending sender, then program order --------- */
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        reinterpret_cast<uint2 *>(s_out[wv])[lane] = make_uint2(o0, o1);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        uint32_t R = 0;                  /* bit 2*sender+word: that word is addressed to me */
        {
            const uint4 *g = reinterpret_cast<const uint4 *>(&s_out[wv][2 * gbase]);
#pragma unroll
            for (int q = 0; q < NP / 2; ++q) {
                const uint4 x = g[q];
                R |= (__builtin_amdgcn_ubfe(x.x, 24 + node, 1) << (4 * q)) |
                     (__builtin_amdgcn_ubfe(x.y, 24 + node, 1) << (4 * q + 1)) |
                     (__builtin_amdgcn_ubfe(x.z, 24 + node, 1) << (4 * q + 2)) |
                     (__builtin_amdgcn_ubfe(x.w, 24 + node, 1) << (4 * q + 3));
            }
        }
        {
            const uint32_t hh = nd.rh & 0xFFu;
            uint32_t cc = nd.rh >> 8;
            bool ovf = false;
            while (R) {
                const uint32_t j = __builtin_ctz(R);
                R &= R - 1;
                const uint32_t x = s_out[wv][2 * gbase + j];
                if (cc < (uint32_t)RING) {
                    s_ring[wv][(hh + cc) & (RING - 1)][lane] = (x & 0x7FFFFFu) | ((j >> 1) << 23);
                    ++cc;
                } else {
                    ovf = true;
                }
            }
            nd.rh = hh | (cc << 8);
            if (ovf) nd.ctl |= C_OVF;
            rmsg = s_ring[wv][hh][lane];          /* next round's head, prefetched */
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");

        /* ---- (5) per-system termination (Appendix A step 4) -------------------------- */
        const uint64_t actb = __ballot(op != OP_IDLE);
        const uint64_t badb = __ballot(live && (nd.ctl & (C_ASSERT | C_OVF)));
        const uint32_t gact = (uint32_t)(actb >> gbase) & NPM;
        const bool gbad = ((badb >> gbase) & NPM) != 0;
        if (live && gact) ++rounds;
        const bool done = live && (gact == 0 || gbad || rounds >= DSM_MAX_ROUNDS);

        const uint64_t doneb = __ballot(done);
        if (doneb) {
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
                const bool handoff = (st == DSM_RING_OVERFLOW) && A.ovf_list;
                const uint32_t fl = ((nd.ctl & C_WAIT) ? 1u : 0u) | ((nd.ctl & C_DUMPED) ? 2u : 0u);
                uint64_t fh = node_hash<16>(node, nd, fl);
                if (A.snap && !handoff) store_rec(&A.snap_final[sys * NP + node], nd, fl);
                fh = gsum64<NP>(fh);
                const uint64_t dh = gsum64<NP>(nd.dh);
                const uint32_t ins = gsum32<NP>(nd.ip);
                uint32_t msgs = 0;
#pragma unroll
                for (uint32_t k = 0; k < 7; ++k) msgs += (nd.tc[k] & 0xFFFFu) + (nd.tc[k] >> 16);
                msgs = gsum32<NP>(msgs);
                uint32_t nlo = 0xFFFFFFFFu, nhi = 0xFFFFFFFFu;
                if (node == 0) {
                    if (handoff) {
                        const uint32_t pos = atomicAdd(A.ovf_count, 1u);
                        A.ovf_list[pos] = (uint32_t)sys;
                        atomicAdd(&s_cnt[wv][K_OVFRERUN], 1ull);
                    } else {
                        if (A.results) {
                            uint4 *rp = reinterpret_cast<uint4 *>(&A.results[sys]);
                            rp[0] = make_uint4(st | (dmask << 8), rounds, msgs, ins);
                            rp[1] = make_uint4((uint32_t)dh, (uint32_t)(dh >> 32), (uint32_t)fh,
                                               (uint32_t)(fh >> 32));
                        }
                        atomicAdd(&s_cnt[wv][K_MSGS], (unsigned long long)msgs);
                        atomicAdd(&s_cnt[wv][K_INSTRS], (unsigned long long)ins);
                        atomicAdd(&s_cnt[wv][K_ROUNDS], (unsigned long long)rounds);
                        atomicAdd(&s_cnt[wv][K_SYSTEMS], 1ull);
                        atomicAdd(&s_cnt[wv][K_STATUS + st], 1ull);
                        atomicAdd(&s_cnt[wv][K_DHASH], (unsigned long long)dh);
                        atomicAdd(&s_cnt[wv][K_FHASH], (unsigned long long)fh);
                        atomicMax(&s_cnt[wv][K_MAXR], (unsigned long long)rounds);
                    }
                    /* next system: static first assignment, then 8 sharded counters */
                    while (tried < 8) {
                        const uint64_t lo = pool + (uint64_t)shard * rs;
                        const uint64_t len = (n > lo) ? ((n - lo) < rs ? (n - lo) : rs) : 0;
                        if (len) {
                            const uint32_t r = atomicAdd(&A.claim[shard * 32u], 1u);
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
                if (!handoff) {
#pragma unroll
                    for (uint32_t t = 0; t < DSM_NTYPES; ++t) {
                        const uint32_t c = (nd.tc[t >> 1] >> ((t & 1u) * 16)) & 0xFFFFu;
                        if (c) atomicAdd(&s_cnt[wv][t], (unsigned long long)c);
                    }
                }
                nlo = __shfl(nlo, (int)gbase, 64);
                nhi = __shfl(nhi, (int)gbase, 64);
                const uint64_t nl = ((uint64_t)nhi << 32) | nlo;
                rounds = 0;
                if (nl != NO_SYS) {
                    sys = A.list ? (uint64_t)A.list[nl] : nl;
                    start_system<NP, GEN>(nd, cur, nxt, tb, sys, node, A);
                } else {
                    live = false;
                }
            }
        }
    }

    /* publish this wave's counters */
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    if (lane < K_N)
        A.partials[((uint64_t)blockIdx.x * WAVES + wv) * K_N + lane] = s_cnt[wv][lane];
}

/* ---- partial-counter reduction (deterministic, one block) ---------------------------- */
__global__ void __launch_bounds__(256) reduce_kernel(const unsigned long long *partials,
                                                     int nwaves, unsigned long long *out) {
    __shared__ unsigned long long s[8][K_N];
    const int k = threadIdx.x & 31, r = threadIdx.x >> 5;
    unsigned long long acc = 0;
    for (int wv = r; wv < nwaves; wv += 8) {
        const unsigned long long x = partials[(size_t)wv * K_N + k];
        acc = (k == K_MAXR) ? (x > acc ? x : acc) : acc + x;
    }
    s[r][k] = acc;
    __syncthreads();
    if (r == 0) {
        for (int i = 1; i < 8; ++i) acc = (k == K_MAXR) ? (s[i][k] > acc ? s[i][k] : acc) : acc + s[i][k];
        out[k] = (k == K_MAXR) ? (acc > out[k] ? acc : out[k]) : out[k] + acc;
    }
}

/* ---- trace generator ------------------------------------------------------------------
 * One workgroup iteration = one (system, node) slot of `stride` instructions; each lane
 * produces 16-byte chunks (8 instructions) and streams them out with non-temporal stores
 * (written once, read later by a different kernel).  No 64-bit divisions in the index math. */
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int NP>
__global__ void __launch_bounds__(256) gen_kernel(uint64_t seed, int dist, uint64_t first,
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
        for (uint32_t k = threadIdx.x; k < cps; k += blockDim.x) {
            u32x4 v;
#pragma unroll
            for (int half = 0; half < 2; ++half) {
                const uint32_t i0 = k * 8 + 4 * half;               /* 4 instructions */
                const uint64_t r = splitmix(base + (i0 >> 2));
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const uint32_t ia = i0 + 2 * j;
                    const uint32_t lo = (ia < n_instr)
                        ? instr_from_bits<NP>((uint32_t)(r >> (32 * j)) & 0xFFFFu, dist) : 0u;
                    const uint32_t hi = (ia + 1 < n_instr)
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
typedef void (*sim_fn)(SimArgs);

template <int NP, bool GEN>
sim_fn fast_kernel(int ring) {
    switch (ring) {
    case 4: return sim_kernel<NP, 4, 4, GEN>;
    case 8: return sim_kernel<NP, 8, 4, GEN>;
    case 32: return sim_kernel<NP, 32, 4, GEN>;
    default: return sim_kernel<NP, 16, 4, GEN>;
    }
}
sim_fn pick_fast(int np, int ring, bool gen) {
    if (np == 4) return gen ? fast_kernel<4, true>(ring) : fast_kernel<4, false>(ring);
    return gen ? fast_kernel<8, true>(ring) : fast_kernel<8, false>(ring);
}
sim_fn pick_fallback(int np, bool gen) {
    if (np == 4) return gen ? sim_kernel<4, 256, 1, true> : sim_kernel<4, 256, 1, false>;
    return gen ? sim_kernel<8, 256, 1, true> : sim_kernel<8, 256, 1, false>;
}

}  // namespace

/* ====================================================================================== */
/* C ABI                                                                                   */
/* ====================================================================================== */

struct dsm_ctx {
    int device;
    dsm_config cfg;
    int ring;
    hipStream_t stream;
    int cus;
    unsigned int *d_ctrl;            /* claim shards (fast, fallback) + overflow count      */
    unsigned long long *d_partials;
    size_t partials_waves;
    uint32_t *d_ovf_list;
    size_t ovf_cap;
    uint16_t *d_traces;
    size_t traces_cap;
    uint32_t *d_counts;
    size_t counts_cap;
    dsm_sys_result *d_res;
    size_t res_cap;
    dsm_counters *d_cnt;
    dsm_node_state *d_snap_dump, *d_snap_final;
    size_t snap_cap_d, snap_cap_f;
    uint64_t snap_n;
    hipEvent_t ev0, ev1;
    int timed;
    dsm_launch_info info;
};

#define CTRL_WORDS 1024
#define CTRL_FAST 0
#define CTRL_FB 256
#define CTRL_OVF 512

#define HIPCK(x) do { if ((x) != hipSuccess) return DSM_E_DEVICE; } while (0)

template <typename T>
static int ensure(T **p, size_t *cap, size_t need) {
    if (*cap >= need && *p) return DSM_OK;
    if (*p) { (void)hipFree(*p); *p = nullptr; *cap = 0; }
    if (hipMalloc((void **)p, need * sizeof(T)) != hipSuccess) { *p = nullptr; return DSM_E_NOMEM; }
    *cap = need;
    return DSM_OK;
}

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
    int ring = cfg->ring_cap ? (int)cfg->ring_cap : 16;
    if (ring != 4 && ring != 8 && ring != 16 && ring != 32) return DSM_E_INVAL;
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
    c->ring = ring;
    c->cus = prop.multiProcessorCount;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc((void **)&c->d_ctrl, CTRL_WORDS * sizeof(unsigned int)) != hipSuccess ||
        hipMalloc((void **)&c->d_cnt, sizeof(dsm_counters)) != hipSuccess) {
        dsm_close(c);
        return DSM_E_DEVICE;
    }
    if ((cfg->flags & DSM_F_TIMING) &&
        (hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess)) {
        dsm_close(c);
        return DSM_E_DEVICE;
    }
    *out = c;
    return DSM_OK;
}

extern "C" void dsm_close(dsm_ctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    void *ptrs[] = {c->d_ctrl, c->d_partials, c->d_ovf_list, c->d_traces, c->d_counts,
                    c->d_res, c->d_cnt, c->d_snap_dump, c->d_snap_final};
    for (void *p : ptrs) if (p) (void)hipFree(p);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    free(c);
}

extern "C" int dsm_launch_info_get(dsm_ctx *c, dsm_launch_info *info) {
    if (!c || !info) return DSM_E_INVAL;
    *info = c->info;
    return DSM_OK;
}

/* Run the transition kernel (+ 256-deep re-run of overflowing systems + counter reduce). */
static int run_engine(dsm_ctx *c, bool gen, const dsm_gen *g, uint64_t first_sys,
                      const uint16_t *d_traces, const uint32_t *d_counts, uint64_t n_sys,
                      dsm_sys_result *d_results, dsm_counters *d_counters, hipStream_t st) {
    if (n_sys == 0) return DSM_OK;
    if (n_sys > 0xFFFFFFFFull) return DSM_E_INVAL;
    HIPCK(hipSetDevice(c->device));
    const int np = c->cfg.np, gpw = 64 / np;
    sim_fn fast = pick_fast(np, c->ring, gen), fb = pick_fallback(np, gen);
    int nb_fast = 0, nb_fb = 0;
    HIPCK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb_fast, (const void *)fast, 256, 0));
    HIPCK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb_fb, (const void *)fb, 64, 0));
    if (nb_fast < 1 || nb_fb < 1) return DSM_E_DEVICE;
    uint64_t want = (n_sys + (uint64_t)(4 * gpw) - 1) / (uint64_t)(4 * gpw);
    int grid_fast = (int)((uint64_t)nb_fast * c->cus < want ? (uint64_t)nb_fast * c->cus : want);
    int grid_fb = nb_fb * c->cus;
    if (grid_fb > 1024) grid_fb = 1024;
    const size_t waves = (size_t)grid_fast * 4 + (size_t)grid_fb;
    int rc;
    if ((rc = ensure(&c->d_partials, &c->partials_waves, waves * K_N))) return rc;
    if ((rc = ensure(&c->d_ovf_list, &c->ovf_cap, (size_t)n_sys))) return rc;
    if (c->cfg.flags & DSM_F_SNAPSHOTS) {
        if ((rc = ensure(&c->d_snap_dump, &c->snap_cap_d, (size_t)n_sys * np))) return rc;
        if ((rc = ensure(&c->d_snap_final, &c->snap_cap_f, (size_t)n_sys * np))) return rc;
        HIPCK(hipMemsetAsync(c->d_snap_dump, 0, (size_t)n_sys * np * sizeof(dsm_node_state), st));
        HIPCK(hipMemsetAsync(c->d_snap_final, 0, (size_t)n_sys * np * sizeof(dsm_node_state), st));
        c->snap_n = n_sys;
    }
    HIPCK(hipMemsetAsync(c->d_ctrl, 0, CTRL_WORDS * sizeof(unsigned int), st));

    SimArgs A;
    memset(&A, 0, sizeof A);
    A.traces = d_traces;
    A.counts = d_counts;
    A.stride = c->cfg.max_instr;
    A.n_instr = gen ? g->n_instr : 0;
    A.n_sys = n_sys;
    A.first_sys = first_sys;
    A.seed = gen ? g->seed : 0;
    A.dist = gen ? g->dist : 0;
    A.snap = (c->cfg.flags & DSM_F_SNAPSHOTS) ? 1 : 0;
    A.results = d_results;
    A.snap_dump = c->d_snap_dump;
    A.snap_final = c->d_snap_final;
    A.partials = c->d_partials;
    A.claim = c->d_ctrl + CTRL_FAST;
    A.ovf_list = c->d_ovf_list;
    A.ovf_count = c->d_ctrl + CTRL_OVF;
    if (c->ev0) HIPCK(hipEventRecord(c->ev0, st));
    hipLaunchKernelGGL(fast, dim3(grid_fast), dim3(256), 0, st, A);
    HIPCK(hipGetLastError());
    if (c->ev1) { HIPCK(hipEventRecord(c->ev1, st)); c->timed = 1; }

    SimArgs B = A;
    B.d_n = c->d_ctrl + CTRL_OVF;
    B.list = c->d_ovf_list;
    B.partials = c->d_partials + (size_t)grid_fast * 4 * K_N;
    B.claim = c->d_ctrl + CTRL_FB;
    B.ovf_list = nullptr;
    B.ovf_count = nullptr;
    hipLaunchKernelGGL(fb, dim3(grid_fb), dim3(64), 0, st, B);
    HIPCK(hipGetLastError());

    hipLaunchKernelGGL(reduce_kernel, dim3(1), dim3(256), 0, st, c->d_partials, (int)waves,
                       (unsigned long long *)d_counters);
    HIPCK(hipGetLastError());

    c->info.grid_blocks = grid_fast;
    c->info.block_threads = 256;
    c->info.waves_per_cu = nb_fast * 4;
    c->info.cus = c->cus;
    c->info.ring_cap = c->ring;
    c->info.lds_bytes_per_block = 4 * (c->ring * 64 * 4 + 64 * 8 + K_N * 8);
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
    const uint64_t cap = (uint64_t)c->cus * 16;
    if (blocks > cap) blocks = cap;
    if (c->cfg.np == 4)
        hipLaunchKernelGGL(gen_kernel<4>, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                           g->seed, g->dist, first_sys, n_sys, g->n_instr, c->cfg.max_instr, d_traces, d_counts);
    else
        hipLaunchKernelGGL(gen_kernel<8>, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                           g->seed, g->dist, first_sys, n_sys, g->n_instr, c->cfg.max_instr, d_traces, d_counts);
    HIPCK(hipGetLastError());
    return DSM_OK;
}

extern "C" int dsm_last_kernel_ms(dsm_ctx *c, float *ms) {
    if (!c || !ms) return DSM_E_INVAL;
    if (!c->ev0 || !c->timed) return DSM_E_STATE;
    HIPCK(hipEventSynchronize(c->ev1));
    HIPCK(hipEventElapsedTime(ms, c->ev0, c->ev1));
    return DSM_OK;
}

extern "C" int dsm_get_node_state(dsm_ctx *c, uint64_t sys, int node, dsm_node_state *dump,
                                  dsm_node_state *final_state) {
    if (!c || node < 0 || node >= c->cfg.np) return DSM_E_INVAL;
    if (!(c->cfg.flags & DSM_F_SNAPSHOTS) || !c->d_snap_dump) return DSM_E_STATE;
    if (sys >= c->snap_n) return DSM_E_INVAL;
    HIPCK(hipSetDevice(c->device));
    HIPCK(hipStreamSynchronize(c->stream));
    HIPCK(hipDeviceSynchronize());
    const size_t i = (size_t)sys * c->cfg.np + node;
    if (dump) HIPCK(hipMemcpy(dump, c->d_snap_dump + i, sizeof *dump, hipMemcpyDeviceToHost));
    if (final_state) HIPCK(hipMemcpy(final_state, c->d_snap_final + i, sizeof *final_state, hipMemcpyDeviceToHost));
    return DSM_OK;
}
