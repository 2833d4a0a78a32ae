/*
 * dsm_table.h -- table-driven transition of one node for one lock-step round.
 *
 * Shared by the gfx950 kernel (dsm_engine.hip) and the host (the table builder, and a CPU
 * model used by the tests).  The 13 message handlers of assignment.c (:177-566) and the
 * instruction issue (:590-687) are compiled into a 640-entry micro-op table:
 *
 *   condition vector C (12 bits, per lane):
 *     bit 0 x     = REPLY_RD exclusive flag (msg.bitVector == 2, :245) for REPLY_RD,
 *                   msg.sender == home (:526) for EVICT_SHARED at a non-home node
 *     bit 1 hit   = line->address == msg.address
 *     bits 2-3    = line->state (M=0 E=1 S=2 I=3)
 *     bit 4 home  = threadId == procNodeAddr (:182)
 *     bit 5 atR2  = threadId == msg.secondReceiver (:286, :483)
 *     bit 6 fwd   = findOwner(dirEntry->bitVector) != msg.sender (:215, :410)
 *     bits 7-8    = dirEntry->state (EM=0 S=1 U=2)
 *     bit 9 sSet  = isBitSet(dirEntry->bitVector, msg.sender) (:501, :545)
 *     bit 10/11   = countSharers after clearing the sender == 0 / == 1 (:504-507)
 *   op' = the message type / issue op, with EVICT_SHARED at its home as its own op (17)
 *         and an unsimulatable instruction (home >= np) as ASSERT (18);
 *   each op' reads one contiguous bit-field of C (its class: lo, width), so
 *   index = op' * 32 + bfe(C, lo, width) -- no per-op branch anywhere.
 *
 * An entry (64 bits) says what to do with the cache line, the directory entry, the memory
 * byte, the two outgoing message words (templates whose operands are picked from a few
 * runtime values), waitingForReply, pendingWriteValue and the assert flag; three bits
 * gate parts of it on `line->address == 0xFF`, the only condition left out of C.
 */
#ifndef DSM_TABLE_H
#define DSM_TABLE_H

#include <stdint.h>

#ifdef __HIPCC__
#define DSM_HD __host__ __device__ __forceinline__
#else
#define DSM_HD static inline
#endif

enum : uint32_t {
    DT_RREQ = 0, DT_WREQ = 1, DT_RRD = 2, DT_RWR = 3, DT_RID = 4, DT_INV = 5, DT_UPG = 6,
    DT_WBINV = 7, DT_WBINT = 8, DT_FLUSH = 9, DT_FLINV = 10, DT_EVS = 11, DT_EVM = 12,
    DT_RD = 13, DT_WR = 14, DT_DUMP = 15, DT_IDLE = 16, DT_EVSH = 17, DT_ASSERT = 18,
    DT_NOPS = 20, DT_STRIDE = 32, DT_ENTRIES = DT_NOPS * DT_STRIDE
};
enum : uint32_t { DT_CM = 0, DT_CE = 1, DT_CS = 2, DT_CI = 3 };   /* cacheLineState :17 */
enum : uint32_t { DT_DEM = 0, DT_DS = 1, DT_DU = 2 };             /* directoryEntryState :18 */

/* class of each op' (3 bits each; ops 0-9 in K0, 10-19 in K1) and (lo, width) per class */
/* classes: 0 none, 1 A [hit Ls], 2 B [x hit Ls], 3 C [hit Ls home atR2], 4 D [fwd Ds],
 *          5 E [Ds sSet rem0 rem1] */
#define DT_CLS(op) ((op) == DT_RREQ || (op) == DT_WREQ ? 4u :                              \
                    (op) == DT_RRD || (op) == DT_EVS ? 2u :                                \
                    (op) == DT_FLUSH || (op) == DT_FLINV ? 3u :                            \
                    (op) == DT_UPG || (op) == DT_EVM || (op) == DT_EVSH ? 5u :             \
                    ((op) == DT_RWR || (op) == DT_RID || (op) == DT_INV ||                 \
                     (op) == DT_WBINV || (op) == DT_WBINT || (op) == DT_RD ||              \
                     (op) == DT_WR) ? 1u : 0u)
#define DT_K(op, base) ((uint32_t)DT_CLS((op) + (base)) << (3 * (op)))
#define DT_KCLS0 (DT_K(0,0) | DT_K(1,0) | DT_K(2,0) | DT_K(3,0) | DT_K(4,0) | DT_K(5,0) |     \
                  DT_K(6,0) | DT_K(7,0) | DT_K(8,0) | DT_K(9,0))
#define DT_KCLS1 (DT_K(0,10) | DT_K(1,10) | DT_K(2,10) | DT_K(3,10) | DT_K(4,10) |           \
                  DT_K(5,10) | DT_K(6,10) | DT_K(7,10) | DT_K(8,10) | DT_K(9,10))
#define DT_KLO 0x761010u   /* nibble per class: lo bit of its field in C  */
#define DT_KW 0x535430u    /* nibble per class: width of its field        */

/* entry, low word.  Every multi-way choice is encoded as independent bits, so the datapath
 * is a tree of selects on bit tests (a chain of `x == k` tests would be turned into a
 * switch, i.e. divergent branches). */
#define E_LA (1u << 0)             /* line.address = a                                   */
#define E_LV(x) ((uint32_t)(x) << 1)  /* line.value: 0 keep 1 v 2 pending 3 zero          */
#define E_LS (1u << 3)             /* line.state = E_LSV                                 */
#define E_LSV(x) ((uint32_t)(x) << 4)
#define E_DBAND0 (1u << 6)         /* dir bv = (bv & AND) | OR; AND: 0xFF, or 0 (this),   */
#define E_DBANDS (1u << 7)         /*   or ~(1 << sender) (this)                         */
#define E_DBORS (1u << 8)          /* OR: 1 << sender                                    */
#define E_DBORR (1u << 9)          /* OR: 1 << secondReceiver                            */
#define E_DS (1u << 10)            /* dir state = E_DSV                                  */
#define E_DSV(x) ((uint32_t)(x) << 11)
#define E_MEM (1u << 13)           /* memory[block] = v                                  */
#define E_O0 (1u << 14)            /* first outgoing word                                */
#define E_O0T(t) ((uint32_t)(t) << 15)
#define E_O0LA (1u << 19)          /* its address is line.address (victim), else a       */
#define E_O0P(x) ((uint32_t)(x) << 20) /* payload: 0 zero 1 Mv 2 bv&~sbit 3 line.value     */
#define E_O0RS (1u << 22)          /* r2 field = sender                                  */
#define E_O0RR (1u << 23)          /* r2 field = secondReceiver                          */
#define E_O0X (1u << 24)           /* exclusive flag                                     */
#define E_O0D(x) ((uint32_t)(x) << 25) /* dest: 0 sender 1 owner 2 home(line) 3 new owner  */
                                       /*       4 home|secondReceiver 5 INV mask           */
#define E_O1 (1u << 28)            /* second word (request to home)                      */
#define E_O1V (1u << 29)           /* its payload is v                                   */
#define E_PEND (1u << 30)          /* pendingWriteValue = v                              */
/* entry, high word */
#define E_WSET (1u << 0)           /* waitingForReply = 1                                */
#define E_WCLR (1u << 1)           /* waitingForReply = 0                                */
#define E_ASSERT (1u << 2)
#define E_O0NFF (1u << 3)          /* first word only if line.address != 0xFF            */
#define E_ANFF (1u << 4)           /* assert only if line.address != 0xFF                */
#define E_LINEFF (1u << 5)         /* line + wait effects only if line.address == 0xFF   */
#define E_O1T(t) ((uint32_t)(t) << 8)  /* type of the second word                         */

/* ---- host: table builder ------------------------------------------------------------- */
/* victim of a replacement (handleCacheReplacement :742-773): word 0 = EVICT_* to La's home */
static inline uint32_t dt_victim(uint32_t Ls) {
    return E_O0 | E_O0NFF | E_O0LA | E_O0D(2) |
           ((Ls == DT_CM) ? (E_O0T(DT_EVM) | E_O0P(3)) : E_O0T(DT_EVS));
}

#define DB_SBIT (E_DBAND0 | E_DBORS)   /* bv = 1 << sender */

static inline void dt_entry(uint32_t opx, uint32_t sub, uint32_t *lo_out, uint32_t *hi_out) {
    const uint32_t cls = (opx < 10) ? ((DT_KCLS0 >> (3 * opx)) & 7u)
                                    : ((DT_KCLS1 >> (3 * (opx - 10))) & 7u);
    const uint32_t lo = (DT_KLO >> (4 * cls)) & 15u, w = (DT_KW >> (4 * cls)) & 15u;
    const uint32_t C = (w ? (sub & ((1u << w) - 1u)) : 0u) << lo;
    const int x = C & 1, hit = (C >> 1) & 1, home = (C >> 4) & 1, atR2 = (C >> 5) & 1;
    const int fwd = (C >> 6) & 1, sSet = (C >> 9) & 1, rem0 = (C >> 10) & 1, rem1 = (C >> 11) & 1;
    const uint32_t Ls = (C >> 2) & 3u, Ds = (C >> 7) & 3u;
    const int valid = Ls != DT_CI, hitv = hit && valid;
    uint32_t e = 0, h = 0;
    switch (opx) {
    case DT_RREQ:                                                     /* :188-236 */
        if (Ds == DT_DU) e = DB_SBIT | E_DS | E_DSV(DT_DEM) | E_O0 | E_O0T(DT_RRD) | E_O0P(1) | E_O0X | E_O0D(0);
        else if (Ds == DT_DS) e = E_DBORS | E_O0 | E_O0T(DT_RRD) | E_O0P(1) | E_O0D(0);
        else if (Ds == DT_DEM && !fwd) e = E_O0 | E_O0T(DT_RRD) | E_O0P(1) | E_O0X | E_O0D(0);
        else if (Ds == DT_DEM) e = E_O0 | E_O0T(DT_WBINT) | E_O0RS | E_O0D(1) | E_DBORS | E_DS | E_DSV(DT_DS);
        break;
    case DT_WREQ:                                                     /* :375-435 */
        e = E_MEM;
        if (Ds == DT_DU) e |= DB_SBIT | E_DS | E_DSV(DT_DEM) | E_O0 | E_O0T(DT_RWR) | E_O0D(0);
        else if (Ds == DT_DS) e |= E_O0 | E_O0T(DT_RID) | E_O0P(2) | E_O0D(0) | DB_SBIT | E_DS | E_DSV(DT_DEM);
        else if (Ds == DT_DEM && !fwd) e |= E_O0 | E_O0T(DT_RWR) | E_O0D(0);
        else if (Ds == DT_DEM) e |= E_O0 | E_O0T(DT_WBINV) | E_O0RS | E_O0D(1) | DB_SBIT;
        break;
    case DT_RRD:                                                      /* :238-247 */
        if (!hit && valid) e |= dt_victim(Ls);
        e |= E_LA | E_LV(1) | E_LS | E_LSV(x ? DT_CE : DT_CS);
        h |= E_WCLR;
        break;
    case DT_RWR:                                                      /* :437-449 */
        e = E_LA | E_LV(2) | E_LS | E_LSV(DT_CM);
        h = E_WCLR;
        if (!hit && valid) h |= E_ASSERT | E_ANFF | E_LINEFF;         /* assert :443 */
        break;
    case DT_RID:                                                      /* :330-364 */
        if (hit) {
            if (Ls != DT_CM) e |= E_LV(2) | E_LS | E_LSV(DT_CM);
            e |= E_O0 | E_O0T(DT_INV) | E_O0D(5);
        }
        h = E_WCLR;
        break;
    case DT_INV:                                                      /* :366-373 */
        if (hit && (Ls == DT_CS || Ls == DT_CE)) e = E_LS | E_LSV(DT_CI);
        break;
    case DT_UPG:                                                      /* :298-328 */
        e = E_O0 | E_O0T(DT_RID) | E_O0D(0) | DB_SBIT | E_DS | E_DSV(DT_DEM) |
            ((Ds == DT_DS) ? E_O0P(2) : 0u);
        break;
    case DT_WBINV:                                                    /* :451-473 */
    case DT_WBINT:                                                    /* :249-271 */
        if (hit && (Ls == DT_CM || Ls == DT_CE))
            e = E_O0 | E_O0T(opx == DT_WBINT ? DT_FLUSH : DT_FLINV) | E_O0P(3) | E_O0RR |
                E_O0D(4) | E_LS | E_LSV(opx == DT_WBINT ? DT_CS : DT_CI);
        break;
    case DT_FLUSH:                                                    /* :273-296 */
        if (home) e |= E_MEM;
        if (atR2) {
            if (!hit && valid) e |= dt_victim(Ls);
            e |= E_LA | E_LV(1) | E_LS | E_LSV(DT_CS);
            h |= E_WCLR;
        }
        break;
    case DT_FLINV:                                                    /* :475-496 */
        if (home) e |= E_MEM | E_DBAND0 | E_DBORR | E_DS | E_DSV(DT_DEM);
        if (atR2) {
            e |= E_LA | E_LV(1) | E_LS | E_LSV(DT_CM);
            h |= E_WCLR;
            if (!hit && valid) h |= E_ASSERT | E_ANFF | E_LINEFF;     /* assert :489 */
        }
        break;
    case DT_EVS:                                                      /* :522-538 */
        if (x && hit && Ls == DT_CS) e = E_LS | E_LSV(DT_CE);
        break;
    case DT_EVSH:                                                     /* :499-521 */
        if (sSet) {
            e = E_DBANDS;
            if (rem0) e |= E_DS | E_DSV(DT_DU);
            else if (rem1 && Ds == DT_DS) e |= E_DS | E_DSV(DT_DEM) | E_O0 | E_O0T(DT_EVS) | E_O0D(3);
        }
        break;
    case DT_EVM:                                                      /* :541-561 */
        e = E_MEM;
        if (Ds == DT_DEM && sSet) e |= E_DBAND0 | E_DS | E_DSV(DT_DU);
        break;
    case DT_RD:                                                       /* :607-630 */
        if (!hitv) {
            if (valid) e |= dt_victim(Ls);
            e |= E_O1 | E_LA | E_LV(3) | E_LS | E_LSV(DT_CI);
            h |= E_WSET | E_O1T(DT_RREQ);
        }
        break;
    case DT_WR:                                                       /* :632-685 */
        e = E_PEND;
        if (hitv) {
            e |= E_LV(1) | E_LS | E_LSV(DT_CM);
            if (Ls == DT_CS) { e |= E_O1; h |= E_WSET | E_O1T(DT_UPG); }
        } else {
            if (valid) e |= dt_victim(Ls);
            e |= E_O1 | E_O1V | E_LA | E_LV(3) | E_LS | E_LSV(DT_CI);
            h |= E_WSET | E_O1T(DT_WREQ);
        }
        break;
    case DT_ASSERT:
        h = E_ASSERT;
        break;
    default:                                                          /* DUMP, IDLE */
        break;
    }
    (void)x;
    *lo_out = e;
    *hi_out = h;
}

/* the whole table: tab[2 * i] = low word, tab[2 * i + 1] = high word */
static inline void dt_build(uint32_t *tab) {
    for (uint32_t op = 0; op < DT_NOPS; ++op)
        for (uint32_t sub = 0; sub < DT_STRIDE; ++sub)
            dt_entry(op, sub, &tab[2 * (op * DT_STRIDE + sub)], &tab[2 * (op * DT_STRIDE + sub) + 1]);
}

/* ---- the datapath (host + device) ----------------------------------------------------- */
struct DtIn {
    uint32_t op;          /* message type 0..12, DT_RD, DT_WR, DT_DUMP or DT_IDLE           */
    uint32_t a, v, r2, s, excl;        /* decoded message / instruction word             */
    uint32_t node, np_mask;
    uint32_t La, Lv, Ls;               /* line at a % 4                                   */
    uint32_t Db, Ds, Mv;               /* directory entry / memory byte at a & 15         */
    uint32_t pend;
};
struct DtOut {
    uint32_t nLa, nLv, nLs, nDb, nDs, nMv;
    uint32_t o0, o1;                   /* outgoing words: body | destination mask << 24   */
    bool wset, wclr;                   /* waitingForReply := 1 / := 0                     */
    bool pendw;                        /* pendingWriteValue := v                          */
    bool asrt;
};

DSM_HD uint32_t dt_index(const DtIn &in, uint32_t *evDb_out, uint32_t *own_out) {
    const uint32_t H = in.a >> 4;
    const uint32_t home = (H == in.node), hit = (in.La == in.a);
    const uint32_t sbit = 1u << in.s;
    const uint32_t ob = in.Db & in.np_mask;
    const uint32_t own = (uint32_t)__builtin_ctz(ob | 0x80000000u);           /* findOwner */
    const uint32_t evDb = in.Db & ~sbit;
    const uint32_t rem = (uint32_t)__builtin_popcount(evDb & in.np_mask);    /* countSharers */
    uint32_t opx = in.op;
    opx = (opx == DT_EVS && home) ? DT_EVSH : opx;
    opx = ((opx == DT_RD || opx == DT_WR) && !((in.np_mask >> H) & 1u)) ? DT_ASSERT : opx;  /* :602 */
    const uint32_t x = (in.op == DT_EVS) ? (uint32_t)(in.s == H) : in.excl;
    const uint32_t C = x | (hit << 1) | (in.Ls << 2) | (home << 4) | ((uint32_t)(in.node == in.r2) << 5) |
                       ((uint32_t)(own != in.s) << 6) | (in.Ds << 7) | (((in.Db >> in.s) & 1u) << 9) |
                       ((uint32_t)(rem == 0) << 10) | ((uint32_t)(rem == 1) << 11);
    const uint32_t cls = (opx < 10) ? ((DT_KCLS0 >> (3 * opx)) & 7u)
                                    : ((DT_KCLS1 >> (3 * (opx - 10))) & 7u);
    const uint32_t lo = (DT_KLO >> (4 * cls)) & 15u, w = (DT_KW >> (4 * cls)) & 15u;
    const uint32_t sub = w ? ((C >> lo) & ((1u << w) - 1u)) : 0u;
    *evDb_out = evDb;
    *own_out = own;
    return opx * DT_STRIDE + sub;
}

DSM_HD DtOut dt_apply(const DtIn &in, uint32_t E0, uint32_t E1, uint32_t evDb, uint32_t own) {
    DtOut o;
    const uint32_t H = in.a >> 4, sbit = 1u << in.s;
    const bool laFF = (in.La == 0xFFu);
    const bool lineOn = !(E1 & E_LINEFF) || laFF;
    /* cache line */
    o.nLa = (lineOn && (E0 & E_LA)) ? in.a : in.La;
    const bool lv0 = lineOn && (E0 & E_LV(1)), lv1 = lineOn && (E0 & E_LV(2));
    o.nLv = lv1 ? (lv0 ? 0u : in.pend) : (lv0 ? in.v : in.Lv);
    o.nLs = (lineOn && (E0 & E_LS)) ? ((E0 >> 4) & 3u) : in.Ls;
    /* directory entry: bv = (bv & AND) | OR */
    const uint32_t andm = (E0 & E_DBANDS) ? ~sbit : (E0 & E_DBAND0) ? 0u : 0xFFu;
    const uint32_t orm = ((E0 & E_DBORS) ? sbit : 0u) | ((E0 & E_DBORR) ? (1u << in.r2) : 0u);
    o.nDb = (in.Db & andm & 0xFFu) | orm;
    o.nDs = (E0 & E_DS) ? ((E0 >> 11) & 3u) : in.Ds;
    o.nMv = (E0 & E_MEM) ? in.v : in.Mv;
    /* first outgoing word */
    const bool p0 = E0 & E_O0P(1), p1 = E0 & E_O0P(2);
    const uint32_t pay = p1 ? (p0 ? in.Lv : (evDb & 0xFFu)) : (p0 ? in.Mv : 0u);
    const uint32_t r2f = (E0 & E_O0RS) ? in.s : (E0 & E_O0RR) ? in.r2 : 0u;
    const bool d0 = E0 & E_O0D(1), d1 = E0 & E_O0D(2), d2 = E0 & E_O0D(4);
    const uint32_t ctzEv = (uint32_t)__builtin_ctz((evDb & in.np_mask) | 0x80000000u);
    const uint32_t didx = d1 ? (d0 ? ctzEv : (in.La >> 4)) : (d0 ? own : in.s);
    const uint32_t mset = d0 ? (in.v & in.np_mask & ~(1u << in.node)) : ((1u << H) | (1u << in.r2));
    const uint32_t dm = d2 ? mset : (1u << didx);
    const bool on0 = (E0 & E_O0) && (!(E1 & E_O0NFF) || !laFF);
    const uint32_t addr0 = (E0 & E_O0LA) ? in.La : in.a;
    o.o0 = on0 ? (((E0 >> 15) & 15u) | (addr0 << 4) | (pay << 11) | (r2f << 19) |
                  (((E0 >> 24) & 1u) << 22) | (dm << 24)) : 0u;
    /* second outgoing word: the request to the home */
    o.o1 = (E0 & E_O1) ? (((E1 >> 8) & 15u) | (in.a << 4) | (((E0 & E_O1V) ? in.v : 0u) << 11) |
                          (1u << (24 + H))) : 0u;
    o.wset = lineOn && (E1 & E_WSET);
    o.wclr = lineOn && (E1 & E_WCLR);
    o.pendw = (E0 & E_PEND) != 0u;
    o.asrt = (E1 & E_ASSERT) && (!(E1 & E_ANFF) || !laFF);
    return o;
}

#endif
