/*
 * dsm_table.h -- table-driven transition of one node for one lock-step round.
 *
 * Shared by the gfx950 kernel (dsm_engine.hip) and the host (the table builder, and a CPU
 * model used by the tests).  The 13 message handlers of assignment.c (:177-566) and the
 * instruction issue (:590-687) are compiled into a 640-entry micro-op table:
 *
 *   condition vector C (11 bits, per lane):
 *     bit 0 x     = the word's exclusive flag: REPLY_RD exclusive (msg.bitVector == 2,
 *                   :245); for EVICT_SHARED at a non-home node msg.sender == home (:526),
 *                   which its only sender (the home, EVICT_SHARED handler :515) sets;
 *                   the WR flag of an issued instruction (RD and WR are one op', DT_RD)
 *     bit 1 hit   = line->address == msg.address
 *     bits 2-3    = line->state (M=0 E=1 S=2 I=3)
 *     bit 4 home  = threadId == procNodeAddr (:182)
 *     bit 5 atR2  = threadId == msg.secondReceiver (:286, :483)
 *     bits 6-7    = dirEntry->state (EM=0 S=1 U=2)
 *     bit 8 sSet  = isBitSet(dirEntry->bitVector, msg.sender) (:501, :545); in state EM the
 *                   bitVector holds exactly one bit, so findOwner(bv) != msg.sender (:215,
 *                   :410) is !sSet (tests/model/table_model.cpp checks the invariant)
 *     bits 9-10   = countSharers after clearing the sender: 0, 1 or 2 = more (:504-507)
 *   op' = the message type / issue op, with EVICT_SHARED at its home as its own op (17)
 *         and an unsimulatable instruction (home >= np) as ASSERT (18);
 *   each op' reads one contiguous bit-field of C (its class: lo, width; a byte per op' in
 *   the table's header, dt_hdr, with the op's first row), so index = base(op') +
 *   bfe(C, lo, width) -- no per-op branch anywhere.  The rows are packed: an op reading a
 *   w-bit field owns 2^w rows (268 rows in all).
 *
 * An entry (64 bits) says what to do with the cache line, the directory entry, the memory
 * byte, the two outgoing message words (templates whose operands are picked from a few
 * runtime values), waitingForReply, pendingWriteValue and the assert flag; a few bits
 * gate parts of it on `line->address == 0xFF`, the only condition left out of C.
 * dt_entry states each handler as micro-op bits (E_*); dt_compile turns them into what the
 * datapath reads: a byte-permute selector (W0) for the four byte results and packed fields
 * (W1).
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
    DT_NOPS = 20, DT_STRIDE = 32,
    DT_ENTRIES = 272,                       /* row capacity (dt_build packs 268 rows)      */
    DT_HDR_WORDS = 64, DT_TABLE_WORDS = 2 * DT_ENTRIES + DT_HDR_WORDS
};
enum : uint32_t { DT_CM = 0, DT_CE = 1, DT_CS = 2, DT_CI = 3 };   /* cacheLineState :17 */
enum : uint32_t { DT_DEM = 0, DT_DS = 1, DT_DU = 2 };             /* directoryEntryState :18 */

/* class of each op' (3 bits each; ops 0-9 in K0, 10-19 in K1) and (lo, width) per class */
/* classes: 0 none, 1 A [hit Ls], 2 B [x hit Ls], 3 C [hit Ls home atR2], 4 D [Ds sSet],
 *          5 E [Ds sSet rem] */
#define DT_CLS(op) ((op) == DT_RREQ || (op) == DT_WREQ ? 4u :                              \
                    (op) == DT_RRD || (op) == DT_EVS || (op) == DT_RD ? 2u :               \
                    (op) == DT_FLUSH || (op) == DT_FLINV ? 3u :                            \
                    (op) == DT_UPG || (op) == DT_EVM || (op) == DT_EVSH ? 5u :             \
                    ((op) == DT_RWR || (op) == DT_RID || (op) == DT_INV ||                 \
                     (op) == DT_WBINV || (op) == DT_WBINT) ? 1u : 0u)
#define DT_K(op, base) ((uint32_t)DT_CLS((op) + (base)) << (3 * (op)))
#define DT_KCLS0 (DT_K(0,0) | DT_K(1,0) | DT_K(2,0) | DT_K(3,0) | DT_K(4,0) | DT_K(5,0) |     \
                  DT_K(6,0) | DT_K(7,0) | DT_K(8,0) | DT_K(9,0))
#define DT_KCLS1 (DT_K(0,10) | DT_K(1,10) | DT_K(2,10) | DT_K(3,10) | DT_K(4,10) |           \
                  DT_K(5,10) | DT_K(6,10) | DT_K(7,10) | DT_K(8,10) | DT_K(9,10))
#define DT_KLO 0x661010u   /* nibble per class: lo bit of its field in C  */
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
    const int sSet = (C >> 8) & 1, fwd = !sSet;
    const int rem0 = ((C >> 9) & 3u) == 0, rem1 = ((C >> 9) & 3u) == 1;
    const uint32_t Ls = (C >> 2) & 3u, Ds = (C >> 6) & 3u;
    const int valid = Ls != DT_CI, hitv = hit && valid;
    uint32_t e = 0, h = 0;
    switch ((opx == DT_RD && x) ? DT_WR : opx) {
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
            else if (rem1 && Ds == DT_DS)       /* the EVICT_SHARED comes from the home: x */
                e |= E_DS | E_DSV(DT_DEM) | E_O0 | E_O0T(DT_EVS) | E_O0X | E_O0D(3);
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
    *lo_out = e;
    *hi_out = h;
}

/* ---- compiled entry: what the datapath reads ------------------------------------------
 * W0 is a v_perm_b32 selector over the candidate bytes
 *     X = {a, v, La, Lv} (bytes 0-3),  Y = {pend, Mv, Db, Db & ~sbit} (bytes 4-7), 12 = 0x00
 * producing the bytes {new line.address, new line.value, new memory byte, first word's
 * payload} in one instruction.  W1 holds the remaining fields (layout below).           */
enum : uint32_t {
    DP_A = 0, DP_V = 1, DP_LA = 2, DP_LV = 3, DP_PEND = 4, DP_MV = 5, DP_DB = 6, DP_EVDB = 7,
    DP_ZERO = 12
};
#define W1_LSEL(x) ((uint32_t)(x) << 0)    /* line.state: selector 0 keep, 4 + k state k     */
#define W1_ORS (1u << 3)                   /* dir bv |= 1 << sender                          */
#define W1_ORR (1u << 4)                   /* dir bv |= 1 << secondReceiver                  */
#define W1_DBASE(x) ((uint32_t)(x) << 5)   /* dir bv base: 0 bv, 1 bv & ~sbit, 2 zero        */
#define W1_O0 (1u << 7)                    /* first word                                     */
#define W1_O1V (1u << 8)                   /* second word's payload is v                     */
#define W1_O0LA (1u << 9)                  /*   address = line.address (victim), else a;
                                            *   bit 9 of a byte-permute selector: byte 2 (La)
                                            *   instead of byte 0 (a)                         */
#define W1_DEST(x) ((uint32_t)(x) << 10)   /*   destination code (E_O0D)                     */
#define W1_R2S (1u << 13)                  /*   secondReceiver field = sender                */
#define W1_R2R (1u << 14)                  /*   secondReceiver field = secondReceiver        */
#define W1_X (1u << 15)                    /*   exclusive flag  } at their places in the     */
#define W1_T(t) ((uint32_t)(t) << 16)      /*   type (4 bits)   } message word               */
#define W1_WSET (1u << 20)
#define W1_WCLR (1u << 21)
#define W1_PEND (1u << 22)
#define W1_ASSERT (1u << 23)
#define W1_DSEL(x) ((uint32_t)(x) << 24)   /* dir state: selector 1 keep, 4 + k state k      */
#define W1_O1(x) ((uint32_t)(x) << 27)     /* second word: 0 none, 1 RREQ, 2 WREQ, 3 UPGRADE  */
#define W1_BSEL(x) ((uint32_t)(x) << 29)   /* the dir bv base again, as a byte-permute selector
                                            * over {0 (bytes 4-7), Y (bytes 0-3)}: 2 Db, 3 Db &
                                            * ~sbit, 4 zero -- one v_perm_b32 (DT_BSEL)       */

/* The 0xFF gates of dt_entry are resolved here.  A line leaves INVALID only by being filled
 * (line.address = a <= 0x7F), and line.address never returns to 0xFF, so a valid line never
 * has address 0xFF: the victim word (handleCacheReplacement :742-745 skips INVALID and 0xFF)
 * is only ever emitted for a valid line, and the REPLY_WR / FLUSH_INVACK asserts (:443,
 * :489), which the table raises only for a valid non-matching line, always fire there,
 * before any line or wait update.  (tests/model/table_model.cpp checks the invariant.)  */
static inline void dt_compile(uint32_t e, uint32_t h, uint32_t *w0, uint32_t *w1) {
    static const uint32_t lv_sel[4] = {DP_LV, DP_V, DP_PEND, DP_ZERO};    /* E_LV codes  */
    static const uint32_t pay_sel[4] = {DP_ZERO, DP_MV, DP_EVDB, DP_LV};  /* E_O0P codes */
    if (h & E_LINEFF) {                                /* the assert fires: no line effects */
        e &= ~(E_LA | E_LV(3) | E_LS | E_LSV(3));
        h &= ~(E_WSET | E_WCLR);
    }
    *w0 = ((e & E_LA) ? DP_A : DP_LA) | (lv_sel[(e >> 1) & 3u] << 8) |
          (((e & E_MEM) ? DP_V : DP_MV) << 16) | (pay_sel[(e >> 20) & 3u] << 24);
    const uint32_t t1 = (h >> 8) & 15u;
    const uint32_t o1 = !(e & E_O1) ? 0u : t1 == DT_RREQ ? 1u : t1 == DT_WREQ ? 2u : 3u;
    *w1 = W1_LSEL((e & E_LS) ? 4u + ((e >> 4) & 3u) : 0u) |
          W1_DSEL((e & E_DS) ? 4u + ((e >> 11) & 3u) : 1u) |
          W1_DBASE((e & E_DBANDS) ? 1u : (e & E_DBAND0) ? 2u : 0u) |
          W1_BSEL((e & E_DBANDS) ? 3u : (e & E_DBAND0) ? 4u : 2u) |
          ((e & E_DBORS) ? W1_ORS : 0u) | ((e & E_DBORR) ? W1_ORR : 0u) |
          ((e & E_O0) ? W1_O0 : 0u) | W1_T((e >> 15) & 15u) | ((e & E_O0LA) ? W1_O0LA : 0u) |
          ((e & E_O0RS) ? W1_R2S : 0u) | ((e & E_O0RR) ? W1_R2R : 0u) | ((e & E_O0X) ? W1_X : 0u) |
          W1_DEST((e >> 25) & 7u) | W1_O1(o1) | ((e & E_O1V) ? W1_O1V : 0u) |
          ((h & E_WSET) ? W1_WSET : 0u) | ((h & E_WCLR) ? W1_WCLR : 0u) |
          ((e & E_PEND) ? W1_PEND : 0u) | ((h & E_ASSERT) ? W1_ASSERT : 0u);
}

/* the whole table, compiled: rows tab[2 * i] = W0, tab[2 * i + 1] = W1, packed op after op
 * (an op with a w-bit field owns 2^w rows), then the header: one word per op',
 * lo | width << 5 | first row << 16 (DT_TABLE_WORDS words in all) */
static inline uint32_t dt_build(uint32_t *tab) {
    for (uint32_t i = 0; i < DT_TABLE_WORDS; ++i) tab[i] = 0;
    uint32_t row = 0;
    for (uint32_t op = 0; op < DT_NOPS; ++op) {
        const uint32_t cls = (op < 10) ? ((DT_KCLS0 >> (3 * op)) & 7u) : ((DT_KCLS1 >> (3 * (op - 10))) & 7u);
        const uint32_t lo = (DT_KLO >> (4 * cls)) & 15u, w = (DT_KW >> (4 * cls)) & 15u;
        tab[2 * DT_ENTRIES + op] = lo | (w << 5) | (row << 16);
        for (uint32_t sub = 0; sub < (1u << w); ++sub, ++row) {
            uint32_t e, h;
            dt_entry(op, sub, &e, &h);
            if (row < DT_ENTRIES) dt_compile(e, h, &tab[2 * row], &tab[2 * row + 1]);
        }
    }
    /* second half, indexed by op | 32 when the message's home is this node: the same
     * headers, with EVICT_SHARED's at-home op (the kernel indexes the header by
     * op | home << 5 instead of selecting DT_EVSH; dt_opx states the same choice) */
    for (uint32_t op = 0; op < 32; ++op)
        tab[2 * DT_ENTRIES + 32 + op] = tab[2 * DT_ENTRIES + (op == DT_EVS ? (uint32_t)DT_EVSH : op)];
    return row;                                  /* rows used; must not exceed DT_ENTRIES */
}

/* ---- the datapath (host + device) ----------------------------------------------------- */
struct DtIn {
    uint32_t op;          /* message type 0..12, DT_RD (an issued RD or WR), DT_DUMP, DT_IDLE */
    uint32_t a, v, r2, s, excl;        /* decoded message / instruction word             */
    uint32_t node, np_mask;
    uint32_t La, Lv, Ls;               /* line at a % 4                                   */
    uint32_t Db, Ds, Mv;               /* directory entry / memory byte at a & 15         */
    uint32_t pend;
};
struct DtOut {
    uint32_t nLa, nLv, nLs, nDb, nDs, nMv;
    uint32_t P;                        /* bytes nLa, nLv, nMv, payload                    */
    uint32_t S;                        /* bytes nLs, -, -, nDs                            */
    uint32_t o0, o1;                   /* outgoing words: body | destination mask << 24   */
    bool wset, wclr;                   /* waitingForReply := 1 / := 0                     */
    bool pendw;                        /* pendingWriteValue := v                          */
    bool asrt;
    uint32_t cset, cclr;               /* the same as a control-word update               */
};
/* node control word bits touched by cset / cclr (dsm_engine.hip's C_WAIT, C_ASSERT) */
enum : uint32_t { DT_CTL_WAIT = 1u << 8, DT_CTL_ASSERT = 1u << 11 };
static_assert((W1_WSET >> 12) == DT_CTL_WAIT && (W1_ASSERT >> 12) == DT_CTL_ASSERT &&
              (W1_WCLR >> 13) == DT_CTL_WAIT, "W1 control bits");

/* ---- message words ---------------------------------------------------------------------
 * A message word (ring entry, outbox word) is laid out like an issued instruction:
 *   bits 0-7 payload (value), 8-14 address, 15 exclusive flag (REPLY_RD) or the WR flag of
 *   an instruction, 16-19 type, 20-22 secondReceiver, 24-31 sender (ring entry) or
 *   destination mask (outbox word).
 * So an instruction of the packed trace (WR << 15 | address << 8 | value, DSM_PACK_INSTR)
 * becomes a word of type DT_RD by one OR, and the first outgoing word's payload and
 * address bytes come out of one byte permute.                                             */
DSM_HD uint32_t dt_issue_word(uint32_t ins) { return ins | (DT_RD << 16); }
DSM_HD uint32_t dt_type(uint32_t w) { return (w >> 16) & 15u; }
DSM_HD uint32_t dt_ring_entry(uint32_t o, uint32_t sender) { return (o & 0xFFFFFFu) | (sender << 24); }
DSM_HD void dt_decode(uint32_t w, uint32_t *a, uint32_t *v, uint32_t *excl, uint32_t *r2, uint32_t *s) {
    *a = (w >> 8) & 0x7Fu; *v = w & 0xFFu; *excl = (w >> 15) & 1u; *r2 = (w >> 20) & 7u; *s = (w >> 24) & 7u;
}

/* Three-input bitwise function (v_bitop3_b32 on gfx950): bit i of the result is bit
 * (a_i << 2 | b_i << 1 | c_i) of the truth table tt (a = 0xF0, b = 0xCC, c = 0xAA: OR3 is 0xFE,
 * (a & b) | c is 0xEA).  On gfx950 it issues at full rate with VGPR or inline-constant
 * operands, where the v_or3_b32 / v_and_or_b32 the compiler picks for the same expressions
 * issue at half rate (tools/calib/valu_rate.hip); the transition round is bound by its VALU
 * issue, so the datapath's three-way combinations are stated with it (DT_B3). */
#ifndef DT_B3
#define DT_B3 1
#endif
#if defined(__HIP_DEVICE_COMPILE__) && DT_B3
#define dt_b3(a, b, c, tt) __builtin_amdgcn_bitop3_b32((a), (b), (c), (tt))
#else
DSM_HD uint32_t dt_b3(uint32_t a, uint32_t b, uint32_t c, uint32_t tt) {
    uint32_t r = 0;
    for (uint32_t k = 0; k < 8; ++k)
        if ((tt >> k) & 1u)
            r |= ((k & 4u) ? a : ~a) & ((k & 2u) ? b : ~b) & ((k & 1u) ? c : ~c);
    return r;
}
#endif
#define DT_OR3 0xFEu
#ifndef DT_BSEL
#define DT_BSEL 1
#endif

/* bit-field extract; width 0 gives 0 (v_bfe_u32) */
DSM_HD uint32_t dt_ubfe(uint32_t x, uint32_t lo, uint32_t w) {
#ifdef __HIP_DEVICE_COMPILE__
    return __builtin_amdgcn_ubfe(x, lo, w);
#else
    return w ? ((x >> lo) & ((1u << w) - 1u)) : 0u;
#endif
}

/* op': the message type / issue op, EVICT_SHARED at its home as DT_EVSH, an instruction
 * whose home is not simulated as DT_ASSERT (:602) */
DSM_HD uint32_t dt_opx(const DtIn &in) {
    const uint32_t H = in.a >> 4;
    uint32_t opx = in.op;
    opx = (opx == DT_EVS && H == in.node) ? DT_EVSH : opx;
    opx = (opx == DT_RD && !((in.np_mask >> H) & 1u)) ? DT_ASSERT : opx;
    return opx;
}

/* table row of op' (header word hdr = dt_hdr) for this lane's conditions */
DSM_HD uint32_t dt_index(const DtIn &in, uint32_t hdr, uint32_t *evDb_out) {
    const uint32_t H = in.a >> 4;
    const uint32_t home = (H == in.node), hit = (in.La == in.a);
    const uint32_t evDb = in.Db & ~(1u << in.s);
    const uint32_t rem = (uint32_t)__builtin_popcount(evDb & in.np_mask);    /* countSharers */
    const uint32_t C = dt_b3(dt_b3(in.excl, hit << 1, in.Ls << 2, DT_OR3),
                             dt_b3(home << 4, (uint32_t)(in.node == in.r2) << 5, in.Ds << 6, DT_OR3),
                             (dt_ubfe(in.Db, in.s, 1) << 8) | ((rem < 2u ? rem : 2u) << 9), DT_OR3);
    *evDb_out = evDb;
    return (hdr >> 16) + dt_ubfe(C, hdr & 31u, (hdr >> 5) & 7u);
}

/* header word of op' (host side; the kernel reads it from the table's header in LDS) */
static inline uint32_t dt_hdr(const uint32_t *tab, uint32_t opx) { return tab[2 * DT_ENTRIES + opx]; }

/* v_perm_b32: byte i of the result = byte sel_i of {hi (bytes 4-7), lo (bytes 0-3)}; 12 = 0 */
DSM_HD uint32_t dt_perm(uint32_t hi, uint32_t lo, uint32_t sel) {
#ifdef __HIP_DEVICE_COMPILE__
    return __builtin_amdgcn_perm(hi, lo, sel);
#else
    const uint64_t v = ((uint64_t)hi << 32) | lo;
    uint32_t r = 0;
    for (int i = 0; i < 4; ++i) {
        const uint32_t k = (sel >> (8 * i)) & 0xFFu;
        const uint32_t b = k < 8u ? (uint32_t)(v >> (8 * k)) & 0xFFu : (k == 12u ? 0u : 0xFFu);
        r |= b << (8 * i);
    }
    return r;
#endif
}

/* the byte-permute operands: X = {a, v, La, Lv}, Y = {pending, Mv, Db, evDb} (the kernel
 * assembles both from its raw words with two permutes, dt_apply_xy) */
DSM_HD uint32_t dt_x(const DtIn &in) { return in.a | (in.v << 8) | (in.La << 16) | (in.Lv << 24); }
DSM_HD uint32_t dt_y(const DtIn &in, uint32_t evDb) {
    return in.pend | (in.Mv << 8) | (in.Db << 16) | ((evDb & 0xFFu) << 24);
}

DSM_HD DtOut dt_apply_xy(const DtIn &in, uint32_t X, uint32_t Y, uint32_t W0, uint32_t W1, uint32_t evDb) {
    DtOut o;
    const uint32_t H = in.a >> 4, sbit = 1u << in.s;
    /* the four byte results in one byte permute */
    const uint32_t P = dt_perm(Y, X, W0);
    o.P = P;
    o.nLa = P & 0xFFu;
    o.nLv = (P >> 8) & 0xFFu;
    o.nMv = (P >> 16) & 0xFFu;
    /* line and directory states: a permute of {Ls, Ds} and the constants 0..3 */
    const uint32_t S = dt_perm(0x03020100u, in.Ls | (in.Ds << 8), W1 & (W1_LSEL(7) | W1_DSEL(7)));
    o.S = S;
    o.nLs = S & 0xFFu;
    o.nDs = S >> 24;
#if DT_BSEL
    /* the base byte picked from Y = {pend, Mv, Db, Db & ~sbit} by the entry's selector: one
     * half-rate permute where the two-level select took two compares and two selects */
    const uint32_t base = dt_perm(0u, Y, (W1 >> 29) | 0x0C0C0C00u);
#else
    const uint32_t db = (W1 >> 5) & 3u;
    const uint32_t base = (db & 2u) ? 0u : (db ? (evDb & 0xFFu) : in.Db);
#endif
    o.nDb = base | ((W1 & W1_ORS) ? sbit : 0u) | ((W1 & W1_ORR) ? (1u << in.r2) : 0u);
    /* first outgoing word: payload and address bytes by one permute of {P, X} (payload =
     * P byte 3; address = X byte 0 (a) or byte 2 (La), per W1_O0LA at selector bit 9),
     * exclusive flag and type straight from W1, secondReceiver field, destinations */
    const uint32_t lo16 = dt_perm(P, X, 0x0C0C0007u | (W1 & W1_O0LA));
    const uint32_t r2f = ((W1 & W1_R2S) ? in.s : 0u) | ((W1 & W1_R2R) ? in.r2 : 0u);
    const uint32_t dc = (W1 >> 10) & 7u;
    const bool d0 = dc & 1u, d1 = dc & 2u, d2 = dc & 4u;
    const uint32_t ctzEv = (uint32_t)__builtin_ctz((evDb & in.np_mask) | 0x80000000u);
    const uint32_t own = (uint32_t)__builtin_ctz((in.Db & in.np_mask) | 0x80000000u);  /* findOwner */
#if defined(SIM_BF) && (SIM_BF & 2)
    const uint32_t m1s = 0u - (uint32_t)d1;                    /* no branch on d1 */
    const uint32_t didx = ((d0 ? ctzEv : (in.La >> 4)) & m1s) | ((d0 ? own : in.s) & ~m1s);
#else
    const uint32_t didx = d1 ? (d0 ? ctzEv : (in.La >> 4)) : (d0 ? own : in.s);
#endif
    const uint32_t mset = d0 ? (in.v & in.np_mask & ~(1u << in.node)) : ((1u << H) | (1u << in.r2));
    const uint32_t dm = d2 ? mset : (1u << didx);
    /* a word is sent iff its destination mask is non-zero; the body of an unsent word is
     * never read, so both words are computed unconditionally (no branch) */
    o.o0 = lo16 | (W1 & (W1_X | W1_T(15))) | (r2f << 20) | ((dm & (0u - ((W1 >> 7) & 1u))) << 24);
    /* second outgoing word: the request to the home (type RREQ 0 / WREQ 1 / UPGRADE 6) */
    const uint32_t c1 = (W1 >> 27) & 3u;
    o.o1 = (((0x6100u >> (4 * c1)) & 15u) << 16) | (in.a << 8) | ((W1 & W1_O1V) ? in.v : 0u) |
           (c1 ? (1u << (24 + H)) : 0u);
    /* node control word (pending byte, wait bit 8, assert bit 11): ctl' = ctl & ~cclr | cset */
    const uint32_t pm = (W1 & W1_PEND) ? 0xFFu : 0u;
    o.cset = ((W1 >> 12) & (DT_CTL_WAIT | DT_CTL_ASSERT)) | (in.v & pm);   /* WSET, ASSERT */
    /* (the kernel's ctl update, ctl & ~cclr | cset, is one v_bitop3 already) */
    o.cclr = ((W1 >> 13) & DT_CTL_WAIT) | pm;                                /* WCLR        */
    o.wset = (W1 & W1_WSET) != 0u;
    o.wclr = (W1 & W1_WCLR) != 0u;
    o.pendw = (W1 & W1_PEND) != 0u;
    o.asrt = (W1 & W1_ASSERT) != 0u;
    return o;
}
DSM_HD DtOut dt_apply(const DtIn &in, uint32_t W0, uint32_t W1, uint32_t evDb) {
    return dt_apply_xy(in, dt_x(in), dt_y(in, evDb), W0, W1, evDb);
}

#endif
