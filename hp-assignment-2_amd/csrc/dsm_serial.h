/*
 * dsm_serial.h -- the lock-step round taken one node-action at a time: one lane (or one host
 * loop) simulates a whole system.  Used by the resume pass of the two-pass schedule
 * (dsm_engine.hip ser_kernel) and by a host model that checks it against the oracle
 * (tests/model/serial_model.cpp).
 *
 * Why: after a few thousand rounds a C3 system is one surviving node issuing its trace while
 * the others wait forever (the home has no transient states,
 * assignment.c:265-270, :467-472), ~1.3 node-actions per round.  The lock-step kernel runs
 * such a system on 8 lanes of which ~1.3 act; here every lane acts in every iteration.
 *
 * Schedule, restated for one node at a time.  In each round every node
 * takes one action decided from its state at the start of the round (inbox head, else idle
 * if waiting, else issue, else dump once); sends are appended at the end of the round in
 * ascending sender order, then program order.  Nodes are taken in ascending order here and
 * a send is appended to the receiver's inbox at once.  That is the same thing, because
 *   - a node's action reads and writes only its own state (assignment.c :157-697: directory,
 *     memory, cache and control of threadId) and appends to other inboxes (sendMessage
 *     :711-739), so the nodes of one round commute but for those appends;
 *   - the appends reach every receiver in (sender, program order), as at the end of the
 *     round;
 *   - a receiver decides from the inbox it had at the start of the round (mask E): an append
 *     goes to the tail, so the head it pops is the one it had, and a node whose inbox was
 *     empty at the start does not pop what arrived during the round.
 * A round in which no node has an action ends the system (`rounds` counts the active ones).
 *
 * Inboxes (round 3): ONE queue per system, not one per node.  After round 2^10 a C3 system
 * holds at most 3 messages in flight (queued at the round start plus appended during it) in
 * 98.3% of its rounds and at most 8 in 99.4% of systems ever (tools/analyze_tail.c), so the
 * system's 8 inboxes share 8 queue slots in append order; byte n of the ownership masks says
 * which slots hold node n's messages, and node n's head is its first slot in queue order.
 * Slots are taken at the tail (qh + qn) and freed where popped; the head advances over freed
 * slots.  When the slot span is full, or anything is already spilled, an append goes to a
 * per-system spill FIFO (global memory on the device; entries carry their receiver) that
 * refills the slots in order, so every inbox keeps its order: node n's messages in slots are
 * older than its spilled ones, and it pops from the spill only when it has none in a slot.
 * A system holds at most 8 + S_SPILL_CAP = 256 queued messages (MSG_BUFFER_SIZE, :12): no
 * inbox can pass the reference's limit, so the default build keeps no per-node counts (an
 * inbox is non-empty iff its ownership byte is, or its node is in the spill mask).  With an
 * inbox limit below 256 (dsm_set_inbox_limit; the CAP build) the counts are kept and an
 * inbox that would exceed the limit, or 255 messages, ends the system's run here with SR_OVF;
 * so does a full spill in either build: the caller hands the system to the 256-deep re-run
 * from scratch, which reports RING_OVERFLOW exactly (the count here can be one higher than at
 * the end of the round, so that hand-off is conservative).
 *
 * A system's column is 104 words (the per-node queues of round 2 took 33 of its 153): six
 * 64-lane waves fit one CU's LDS, two waves on two of its SIMDs, against four waves (one per
 * SIMD) before -- the iteration is a dependent chain that one wave alone cannot hide.
 */
#ifndef DSM_SERIAL_H
#define DSM_SERIAL_H

#ifndef SER_NOTICE_HOME
#define SER_NOTICE_HOME 1   /* ... and an upgrade notice to either home */
#endif
#ifndef SER_DUMP
#define SER_DUMP 0          /* ... and the lone node's dump (exact, but C5 33.4 vs 32.5 ms: off) */
#endif
#ifndef SER_DEAD_FWD
#define SER_DEAD_FWD 1      /* ser_macro also applies a system's dead-end forward */
#endif

#include "dsm_table.h"

namespace dsms {

/* per-system words (one LDS column per lane on the device, a plain array on the host):
 *   S_MB + 8n + p   node n, blocks 2p and 2p+1: memory | bitVector << 8 per 16-bit half
 *   S_LA + n        node n, cache line addresses, a byte per line
 *   S_LV + n        node n, cache line values, a byte per line
 *   S_DS + n        node n, directory states (2 bits per block)
 *   S_CT + n        node n, control: pendingWriteValue 0-7 | wait 8 | dumped 9 |
 *                   line states 10-17 (2 bits per line) | instructions issued 18-31
 *   S_Q + s         queue slot s: ring entry (body | sender << 24) | receiver << 27     */
enum : uint32_t { S_MB = 0, S_LA = 64, S_LV = 72, S_DS = 80, S_CT = 88, S_Q = 96, S_WORDS = 104 };
constexpr uint32_t S_QN = 8, S_SPILL = 256;      /* queue slots; spill entries per system */
constexpr uint32_t S_SPILL_CAP = 256 - S_QN;     /* used spill entries: 8 + 248 = 256     */
constexpr uint32_t S_TOMB = 0xFFFFFFFFu;         /* a spill entry taken out of order      */

/* control bits (the lock-step kernel's C_*): wait 8, dumped 9; the table's assert bit (11)
 * is taken out of the control word at once (the system ends at the end of the round) */
enum : uint32_t { SC_WAIT = DT_CTL_WAIT, SC_DUMPED = 1u << 9, SC_ASSERT = DT_CTL_ASSERT,
                  SC_LS = 10, SC_IP = 18 };
enum : uint32_t { SR_RUN = 0, SR_DONE = 1, SR_OVF = 2 };          /* ser_step verdicts */
/* statuses (include/dsm.h DSM_*) */
enum : uint32_t { SS_COMPLETED = 0, SS_DEADLOCKED = 1, SS_ASSERT = 3, SS_ROUND_LIMIT = 4 };
constexpr uint32_t S_LA_INIT = 0xFFFFFFFFu;      /* every line: address 0xFF              */
constexpr uint32_t S_LS_INIT = 0xFFu << SC_LS;   /* every line INVALID (3)                */

/* a system's registers */
struct SReg {
    uint32_t A;       /* nodes still to act in this round                                   */
    uint32_t E;       /* nodes whose inbox was non-empty at the start of this round         */
    uint32_t nz;      /* nodes whose inbox is non-empty now                                 */
    uint32_t iss;     /* nodes neither waiting nor dumped: they issue, or dump, next        */
    uint32_t dmp;     /* nodes that dumped                                                   */
    uint32_t own0, own1;   /* bit s of byte n: slot s holds a message for node n (0-3, 4-7)   */
    uint32_t cnt0, cnt1;   /* CAP build: inbox counts (slots + spill), a byte per node       */
    uint32_t spl;     /* nodes with a message in the spill                                  */
    uint32_t L;       /* slots holding a message                                            */
    uint32_t q;       /* qh 0-2 | qn 3-6 (slots from qh to the tail) | sq 7-15 (spill
                       * entries, taken ones included) | sh 16-23 (spill head)             */
    uint32_t ni01, ni23, ni45, ni67;   /* instructions in each node's trace, 16 bits each  */
    uint32_t rounds;  /* active rounds                                                      */
    uint32_t msgs;    /* messages handled                                                   */
    uint32_t asrt;    /* an assert fired in this round                                      */
    uint32_t st;      /* status once SR_DONE                                                */
};

DSM_HD uint32_t s_ctz(uint32_t x) { return (uint32_t)__builtin_ctz(x); }
/* some lane of the wave has c (the host model's one "lane": c) -- a wave-uniform branch
 * around a load that most lanes take from registers (an LDS read under a per-lane select is
 * issued for every lane and waited for on the chain) */
DSM_HD bool s_any(bool c) {
#ifdef __HIP_DEVICE_COMPILE__
    return __ballot(c) != 0ull;
#else
    return c;
#endif
}
/* b where bit k of n is set, else a -- by masks (v_bfi): a `?:` of two members of the
 * register struct is turned into a load from a selected address, which puts the whole
 * struct in scratch memory */
DSM_HD uint32_t s_pick(uint32_t a, uint32_t b, uint32_t n, uint32_t k) {
    const uint32_t m = 0u - ((n >> k) & 1u);
    return (a & ~m) | (b & m);
}
/* byte n of the 8-byte value (hi:lo) -- two registers, not an array (an array indexed at
 * run time goes to scratch memory) */
DSM_HD uint32_t s_byte(uint32_t lo, uint32_t hi, uint32_t n) {
    return (s_pick(lo, hi, n, 2) >> (8u * (n & 3u))) & 0xFFu;
}
/* (hi:lo) += x << 8 n (x may be "negative": a wrapped subtraction inside the byte) */
DSM_HD void s_byte_add(uint32_t &lo, uint32_t &hi, uint32_t n, uint32_t x) {
    const uint32_t d = x << (8u * (n & 3u));
    lo += (n & 4u) ? 0u : d;
    hi += (n & 4u) ? d : 0u;
}
DSM_HD uint32_t s_ni(const SReg &r, uint32_t n) {
    const uint32_t w = s_pick(s_pick(r.ni01, r.ni23, n, 1), s_pick(r.ni45, r.ni67, n, 1), n, 2);
    return (w >> (16u * (n & 1u))) & 0xFFFFu;
}
DSM_HD void s_set_ni(SReg &r, uint32_t n, uint32_t v) {   /* selects: no pointer to a member */
    const uint32_t sh = 16u * (n & 1u), k = n >> 1;
    const uint32_t m = ~(0xFFFFu << sh), x = (v & 0xFFFFu) << sh;
    r.ni01 = k == 0u ? ((r.ni01 & m) | x) : r.ni01;
    r.ni23 = k == 1u ? ((r.ni23 & m) | x) : r.ni23;
    r.ni45 = k == 2u ? ((r.ni45 & m) | x) : r.ni45;
    r.ni67 = k == 3u ? ((r.ni67 & m) | x) : r.ni67;
}
DSM_HD uint32_t s_qh(uint32_t q) { return q & 7u; }
DSM_HD uint32_t s_qn(uint32_t q) { return (q >> 3) & 15u; }
DSM_HD uint32_t s_sq(uint32_t q) { return (q >> 7) & 511u; }
DSM_HD uint32_t s_sh(uint32_t q) { return (q >> 16) & 255u; }

/* empty queue, no spill */
DSM_HD void ser_clear(SReg &r) {
    r.A = r.E = r.nz = r.iss = r.dmp = 0;
    r.own0 = r.own1 = r.cnt0 = r.cnt1 = r.spl = r.L = r.q = 0;
    r.ni01 = r.ni23 = r.ni45 = r.ni67 = 0;
    r.rounds = r.msgs = r.asrt = r.st = 0;
}

/* append entry e (ring entry: body | sender << 24) to node d's inbox, at the queue's tail
 * or, when the slot span is full or something is already spilled, to the spill.  Returns
 * false (nothing appended) when the spill is full.  Counts are the caller's. */
template <uint32_t Q, class M>
DSM_HD bool ser_enqueue(M &m, SReg &r, uint32_t d, uint32_t e) {
    const uint32_t qn = s_qn(r.q), sq = s_sq(r.q);
    if (sq == 0u && qn < Q) {
        const uint32_t slot = (s_qh(r.q) + qn) & 7u;
        m.st(S_Q + slot, e | (d << 27));
        r.L |= 1u << slot;
        s_byte_add(r.own0, r.own1, d, 1u << slot);
        r.q += 1u << 3;
        return true;
    }
    if (sq >= S_SPILL_CAP) return false;
    m.sp_st((s_sh(r.q) + sq) & (S_SPILL - 1u), e | (d << 27));
    r.q += 1u << 7;
    r.spl |= 1u << d;
    return true;
}

/* slow paths (rare: more than 8 messages in flight) ---------------------------------------- */
/* the nodes that still have a message in the spill */
template <class M>
DSM_HD uint32_t ser_spill_nodes(M &m, const SReg &r) {
    const uint32_t sq = s_sq(r.q), sh = s_sh(r.q);
    uint32_t spl = 0;
    for (uint32_t i = 0; i < sq; ++i) {
        const uint32_t v = m.sp_ld((sh + i) & (S_SPILL - 1u));
        spl |= v != S_TOMB ? 1u << ((v >> 27) & 7u) : 0u;
    }
    return spl;
}
/* node n has no message in a slot: its head is its first entry in the spill; take it out
 * (a tombstone), then drop leading tombstones */
template <class M>
DSM_HD uint32_t ser_spill_take(M &m, SReg &r, uint32_t n) {
    const uint32_t sq = s_sq(r.q), sh = s_sh(r.q);
    uint32_t e = 0;
    for (uint32_t i = 0; i < sq; ++i) {
        const uint32_t ix = (sh + i) & (S_SPILL - 1u);
        const uint32_t v = m.sp_ld(ix);
        if (v != S_TOMB && (v >> 27) == n) {
            e = v;
            m.sp_st(ix, S_TOMB);
            break;
        }
    }
    uint32_t h = sh, c = sq;
    while (c != 0u && m.sp_ld(h) == S_TOMB) { h = (h + 1u) & (S_SPILL - 1u); --c; }
    r.q = (r.q & 0xFF00007Fu) | (c << 7) | (h << 16);
    r.spl = ser_spill_nodes(m, r);
    return e;
}
/* refill free tail slots from the spill, in order (skipping tombstones) */
template <uint32_t Q, class M>
DSM_HD void ser_refill(M &m, SReg &r) {
    uint32_t qh = s_qh(r.q), qn = s_qn(r.q), sq = s_sq(r.q), sh = s_sh(r.q);
    while (qn < Q && sq != 0u) {
        const uint32_t v = m.sp_ld(sh);
        sh = (sh + 1u) & (S_SPILL - 1u);
        --sq;
        if (v == S_TOMB) continue;
        const uint32_t slot = (qh + qn) & 7u;
        m.st(S_Q + slot, v);
        r.L |= 1u << slot;
        s_byte_add(r.own0, r.own1, v >> 27, 1u << slot);
        ++qn;
    }
    r.q = qh | (qn << 3) | (sq << 7) | (sh << 16);
    r.spl = ser_spill_nodes(m, r);
}

/* a fresh system: initializeProcessor :778-790 and main :142-146 for every node */
template <int NP, class M>
DSM_HD void ser_fresh(M &m, SReg &r, const uint32_t *counts, uint32_t stride) {
    ser_clear(r);
    for (uint32_t n = 0; n < (uint32_t)NP; ++n) {
        for (uint32_t p = 0; p < 8; ++p)
            m.st(S_MB + 8 * n + p, ((20u * n + 2 * p) & 0xFFu) | (((20u * n + 2 * p + 1) & 0xFFu) << 16));
        m.st(S_LA + n, S_LA_INIT);
        m.st(S_LV + n, 0u);
        m.st(S_DS + n, 0xAAAAAAAAu);                       /* every block UNOWNED */
        m.st(S_CT + n, S_LS_INIT);
        s_set_ni(r, n, counts[n] < stride ? counts[n] : stride);
    }
    r.A = r.iss = (1u << NP) - 1u;
}

/* one node-action of the system (the lowest node left in this round), then, if it was the
 * round's last, the end of the round.  Branch-free but for the dump record, the rare third-
 * and-later destinations of a multicast and the spill paths: on the device every lane of a
 * wave runs a different system, and divergent branches cost more than the predicated work.
 *   F fetch(node, index, issue) -> the packed instruction (only used when issue);
 *   R on_dump(node): the node's dump record is due (state as stored, flags 2).
 * M: the system's words (ld / st / st_if (a store when the flag is set, else to a dummy
 * word: no branch) / ld8 / st8 / ld16 / st16) and its spill FIFO (sp_ld / sp_st (index),
 * S_SPILL entries).  CAP: the build for an inbox limit below 256 (per-node counts kept).  Q <= 8: the slot span (the kernel's 8; the host model
 * takes fewer to send more systems through the spill). */
template <int NP, uint32_t Q = S_QN, bool CAP = false, class M, class T, class F, class R>
DSM_HD uint32_t ser_step(M &m, SReg &r, const T &tab, F &&fetch, R &&on_dump, uint32_t lim_rsh,
                         uint32_t cap = 256u) {
    constexpr uint32_t NPM = (1u << NP) - 1u;
    const uint32_t n = s_ctz(r.A), bit = 1u << n;
    uint32_t ct = m.ld(S_CT + n);
    const uint32_t nins = s_ni(r, n);
    const bool hasMsg = (r.E & bit) != 0u;                        /* :158-169 */
    /* the inbox head: node n's first slot in queue order from qh (k == 8: none; the head is
     * in the spill) */
    const uint32_t ob = s_byte(r.own0, r.own1, n);
    const uint32_t qh = s_qh(r.q);
    const uint32_t k = s_ctz((((ob | (ob << 8)) >> qh) & 0xFFu) | 0x100u);
    const uint32_t slot = (qh + k) & 7u;
    uint32_t rw = m.ld(S_Q + slot);                               /* (may be stale)     */
    if (hasMsg && k == 8u) rw = ser_spill_take(m, r, n);
    const uint32_t ip = ct >> SC_IP;
    const bool doIssue = !hasMsg && ip < nins;                    /* :590-592 */
    const bool doDump = !hasMsg && !doIssue;                      /* :688-697 */
    const uint32_t ins = fetch(n, ip, doIssue);
    const uint32_t w = hasMsg ? rw : dt_issue_word(ins);
    {   /* pop the head: free its slot, advance the queue head past free slots (branch-free:
         * bit operations and selects; the head moves only when its own slot was popped) */
        const bool popq = hasMsg & (k < 8u);
        const uint32_t sb = popq ? (1u << slot) : 0u;
        s_byte_add(r.own0, r.own1, n, 0u - sb);
        r.L &= ~sb;
        if (CAP) s_byte_add(r.cnt0, r.cnt1, n, hasMsg ? 0xFFFFFFFFu : 0u);
        const bool empty = CAP ? s_byte(r.cnt0, r.cnt1, n) == 0u : ((ob & ~sb) | (r.spl & bit)) == 0u;
        r.nz &= (hasMsg & empty) ? ~bit : ~0u;
        r.msgs += hasMsg ? 1u : 0u;
        const uint32_t qn = s_qn(r.q), L = r.L;
        uint32_t adv = s_ctz((((L | (L << 8)) >> qh) & 0xFFu) | 0x100u);
        adv = adv < qn ? adv : qn;
        adv = (popq & (k == 0u)) ? adv : 0u;
        r.q = (r.q & ~0x7Fu) | ((qh + adv) & 7u) | ((qn - adv) << 3);
        if ((uint32_t)(s_sq(r.q) != 0u) & (uint32_t)(s_qn(r.q) < Q)) ser_refill<Q>(m, r);
    }
    ct += doIssue ? (1u << SC_IP) : 0u;
    const uint32_t op = doDump ? (uint32_t)DT_DUMP : dt_type(w);

    /* decode + micro-op table + datapath (dsm_table.h), as in sim_kernel step (2)-(3) */
    DtIn in;
    dt_decode(w, &in.a, &in.v, &in.excl, &in.r2, &in.s);
    const uint32_t blk = in.a & 15u, idx = in.a & 3u;            /* :177-184 */
    const uint32_t mw = S_MB + 8u * n + (blk >> 1);
    const uint32_t mbw = m.ld16(mw, blk & 1u);
    const uint32_t La = m.ld8(S_LA + n, idx), Lv = m.ld8(S_LV + n, idx);
    const uint32_t dsw = m.ld(S_DS + n);
    const uint32_t lsh = SC_LS + 2u * idx;
    in.op = op; in.node = n; in.np_mask = NPM;
    in.La = La; in.Lv = Lv; in.Ls = dt_ubfe(ct, lsh, 2u);
    in.Db = mbw >> 8; in.Ds = dt_ubfe(dsw, 2u * blk, 2u); in.Mv = mbw & 0xFFu; in.pend = ct & 0xFFu;
    uint32_t hix = op | ((in.a >> 4) == n ? 32u : 0u);
    if (NP < 8) hix = (op == DT_RD && (in.a >> 4) >= (uint32_t)NP) ? (uint32_t)DT_ASSERT : hix;
    uint32_t evDb;
    const uint32_t ti = dt_index(in, tab.hdr(hix), &evDb);
    uint32_t W0, W1;
    tab.row(ti, W0, W1);
    const uint32_t X = dt_perm(La | (Lv << 8), w, 0x05040001u) & ~0x80u;   /* {a, v, La, Lv} */
    const uint32_t Y = dt_perm(mbw, ct, 0x0C050400u) | ((evDb & 0xFFu) << 24);
    const DtOut o = dt_apply_xy(in, X, Y, W0, W1, evDb);
    m.st8(S_LA + n, idx, o.P);                                   /* nLa */
    m.st8(S_LV + n, idx, o.P >> 8);                              /* nLv */
    m.st(S_DS + n, (dsw & ~(3u << (2u * blk))) | (o.nDs << (2u * blk)));
    m.st16(mw, blk & 1u, o.nMv | (o.nDb << 8));
    r.asrt |= o.cset & SC_ASSERT;
    ct = (ct & ~(o.cclr | (3u << lsh))) | (o.cset & ~SC_ASSERT) | (o.nLs << lsh) |
         (doDump ? SC_DUMPED : 0u);                              /* wait, pending (:633) */
    m.st(S_CT + n, ct);
    r.dmp |= doDump ? bit : 0u;
    if (doDump) on_dump(n);                  /* printProcessorState(threadId, node), :695 */
    r.iss = (ct & (SC_WAIT | SC_DUMPED)) ? (r.iss & ~bit) : (r.iss | bit);

    /* sendMessage :711-739: the first word to its destinations in ascending order, then the
     * second; each to the tail of the receiver's inbox */
    bool ovf = false;
    auto append = [&](bool en, uint32_t d, uint32_t e) {
        bool ok = en;
        if (CAP) {
            const uint32_t c = s_byte(r.cnt0, r.cnt1, d);
            const bool over = en & ((c >= cap) | (c >= 255u));
            ok = en & !over;
            ovf = ovf | over;
            s_byte_add(r.cnt0, r.cnt1, d, ok ? 1u : 0u);
        }
        const uint32_t qn = s_qn(r.q);
        const bool fast = ok & ((r.q & 0xFF80u) == 0u) & (qn < Q);     /* no spill, a slot */
        const uint32_t as = (r.q + qn) & 7u;                           /* (qh + qn) & 7    */
        m.st_if(fast, S_Q + as, e | (d << 27));
        const uint32_t sb = fast ? (1u << as) : 0u;
        r.L |= sb;
        s_byte_add(r.own0, r.own1, d, sb);
        r.q += fast ? (1u << 3) : 0u;
        r.nz |= ok ? 1u << d : 0u;
        if (ok & !fast) ovf = !ser_enqueue<Q>(m, r, d, e) || ovf;  /* the spill (rare)   */
    };
    {
        uint32_t dm = o.o0 >> 24;
        const uint32_t e0 = dt_ring_entry(o.o0, n);
        append(dm != 0u, s_ctz(dm | 0x100u) & 7u, e0);          /* first destination  */
        dm &= dm - 1u;
        append(dm != 0u, s_ctz(dm | 0x100u) & 7u, e0);          /* second (FLUSH: home + requester) */
        dm &= dm - 1u;
        while (dm) {                                              /* an INV multicast    */
            append(true, s_ctz(dm), e0);
            dm &= dm - 1u;
        }
        const uint32_t d1 = o.o1 >> 24;
        append(d1 != 0u, s_ctz(d1 | 0x100u) & 7u, dt_ring_entry(o.o1, n));
    }

    /* ---- end of the round (Appendix A step 4) ---- */
    r.A &= ~bit;
    if (ovf) return SR_OVF;
    if (r.A) return SR_RUN;
    r.rounds++;
    if (r.asrt) { r.st = SS_ASSERT; return SR_DONE; }            /* a failed assert */
    if (r.rounds >> lim_rsh) { r.st = SS_ROUND_LIMIT; return SR_DONE; }
    r.E = r.nz;
    r.A = r.nz | r.iss;
    if (r.A == 0u) {                                           /* quiescent */
        r.st = (r.dmp == NPM) ? SS_COMPLETED : SS_DEADLOCKED;
        return SR_DONE;
    }
    return SR_RUN;
}

/* ---- lone-survivor transaction macro-step (round 4) ---------------------------------------
 * After a few thousand rounds a system is one node issuing while every other node waits for
 * good (or has dumped), with nothing queued: 97% (C3) / 99% (C5) of the serial pass's
 * node-actions are that node's whole transactions (tools/analyze_macro.c).  From such a quiet
 * state the schedule is fixed and short: round 1 the node issues; a hit ends there.  A miss
 * sends the victim's EVICT_* (:616-618, :742-773) to the victim's home, then the request to
 * the block's home; in round 2 both are handled (the victim's home first, in the round after
 * when it is also the block's home: its inbox holds the eviction, then the request); the reply
 * is handled in the round after the request.  A write hit on SHARED sends UPGRADE (:646-659)
 * and takes the same three rounds without an eviction.  When the handlers send nothing else
 * -- the eviction's home sends no upgrade notice (:507-519), the request's home answers the
 * requester directly (no WRITEBACK_INT / WRITEBACK_INV to another owner, :210-233,
 * :405-432), and a REPLY_ID names no other sharer (no INV fan-out, :350-362) -- the whole
 * transaction is applied here at once, straight from its handlers:
 *   EVICT_MODIFIED :541-561, EVICT_SHARED :498-539 (at the home), READ_REQUEST :188-236,
 *   WRITE_REQUEST :375-435, UPGRADE :298-328, REPLY_RD :238-247, REPLY_WR :437-449,
 *   REPLY_ID :330-364,
 * with `rounds` and `msgs` advanced as the lock-step schedule would.  The two homes' words
 * are read up front and forwarded when the victim's and the request's blocks share one.
 * fetch(node, index, &ins) -> false when the instruction is not at hand without a memory
 * load (the kernel's register-held trace chunks; ser_step then takes the issue and loads it).
 * Returns false, changing nothing but the fetch cache, when the system is not in such a state
 * or the transaction would send anything else; ser_step then takes it one action at a time.
 * Not used in the CAP build (its per-node inbox counts are not kept here). */
/* the most rounds one ser_macro call adds: the request after an eviction at the same home
 * (3), then a forward and its flush (2).  ser_quiet_lone keeps that many plus the round after
 * (a fan-out's INVs) below the round limit; the host model checks every call's advance
 * against it (tests/model/serial_model.cpp). */
constexpr uint32_t SER_MACRO_MAX_ROUNDS = 5;
DSM_HD bool ser_quiet_lone(const SReg &r, uint32_t lim_rsh) {
    /* nothing queued or spilled, exactly one node may act and it is the only one left in the
     * round, and the round limit is out of reach of the transaction's rounds and the round
     * after */
    return (r.nz | (r.q & 0xFFF8u) | r.spl) == 0u && r.A == r.iss && r.A != 0u && (r.A & (r.A - 1u)) == 0u &&
           ((r.rounds + SER_MACRO_MAX_ROUNDS + 1u) >> lim_rsh) == 0u;
}

/* the lone node's own words (control, line addresses, line values) held in registers
 * between macro-steps: only the node's own actions write them, and a macro-step is the only
 * action of a system between two of them (ser_step or a hand-over invalidates the cache) */
struct SCache {
    uint32_t ct, la, lv, node;      /* node: the node they belong to, 0xFF: none */
};
DSM_HD void ser_cache_clear(SCache &c) { c.ct = c.la = c.lv = 0u; c.node = 0xFFu; }

/* stamp(i): diagnostic hook (the kernel's SER_PROBE 4 build times the step's phases; else a
 * no-op) */
template <int NP, class M, class F, class R, class P>
DSM_HD bool ser_macro(M &m, SReg &r, SCache &cc, F &&fetch, R &&on_dump, P &&stamp) {
    constexpr uint32_t NPM = (1u << NP) - 1u;
    const uint32_t n = s_ctz(r.A), bit = 1u << n;
    const bool hot = cc.node == n;
    uint32_t ct = cc.ct;
    if (s_any(!hot)) {
        const uint32_t x = m.ld(S_CT + n);
        ct = hot ? ct : x;
    }
    const uint32_t ip = ct >> SC_IP;
    if (ip >= s_ni(r, n)) {
        /* the trace is done: the dump (:688-697), the round's one action; then no node can
         * act and the system is quiescent (the caller ends it when r.A is empty) */
        if (!SER_DUMP) return false;
        ct |= SC_DUMPED;
        m.st(S_CT + n, ct);
        r.dmp |= bit;
        on_dump(n);                          /* printProcessorState(threadId, node), :695 */
        r.iss &= ~bit;
        r.A = r.iss;
        r.rounds += 1u;
        r.E = 0u;
        r.st = (r.dmp == NPM) ? SS_COMPLETED : SS_DEADLOCKED;
        cc.ct = ct; cc.node = n;
        return true;
    }
    uint32_t ins;
    if (!fetch(n, ip, ins)) return false;                     /* not at hand: ser_step loads it */
    stamp(0);
    const uint32_t a = (ins >> 8) & 0x7Fu, wr = ins >> 15, val = ins & 0xFFu;
    const uint32_t h = a >> 4, b = a & 15u, idx = a & 3u, sh8 = 8u * idx;
    uint32_t laW = cc.la, lvW = cc.lv;
    if (s_any(!hot)) {
        const uint32_t x = m.ld(S_LA + n), y = m.ld(S_LV + n);
        laW = hot ? laW : x;
        lvW = hot ? lvW : y;
    }
    const uint32_t La = (laW >> sh8) & 0xFFu, Lv = (lvW >> sh8) & 0xFFu;
    const uint32_t lsh = SC_LS + 2u * idx, Ls = (ct >> lsh) & 3u;          /* M0 E1 S2 I3 */
    const bool hit = (La == a) & (Ls != 3u);                   /* :608, :635 */
    const bool upg = hit & (wr != 0u) & (Ls == 2u);            /* write hit on SHARED :646 */
    const bool miss = !hit;
    const bool ev = miss & (La != 0xFFu) & (Ls != 3u);         /* :616-618, :670-672 */
    /* the victim's home vh, block vb; the request's home h, block b (every home < NP: a line
     * holds an address some request brought in; h is checked).  All four words are read at
     * once; the request's home sees the eviction's effect when they share a word.  The
     * victim's line has the same index as the request's (it is the line being replaced). */
    const uint32_t vh = (La >> 4) & 7u, vb = La & 15u;
    const uint32_t wV = S_MB + 8u * vh + (vb >> 1), wH = S_MB + 8u * h + (b >> 1);
    const uint32_t mbV = m.ld(wV), dsV = m.ld(S_DS + vh);
    const uint32_t mbH0 = m.ld(wH), dsH0 = m.ld(S_DS + h);
    /* the eviction at the victim's home (:498-561) */
    const uint32_t hv = 16u * (vb & 1u), sv = 2u * vb;
    const uint32_t memV = (mbV >> hv) & 0xFFu, bvV = (mbV >> (hv + 8u)) & 0xFFu, dV = (dsV >> sv) & 3u;
    stamp(1);
    const bool mod = Ls == 0u;
    const bool had = (bvV & bit) != 0u;
    const uint32_t bvS = bvV & ~bit;                            /* EVICT_SHARED, bit set */
    const uint32_t rem = (uint32_t)__builtin_popcount(bvS);
    /* EVICT_SHARED leaving one sharer x of an S entry: EM {x} and an upgrade notice to x
     * (:507-519), handled by x in round 3 -- x's line, if it still holds the block in S,
     * becomes EXCLUSIVE (:526-532) */
    const bool notice = ev & !mod & had & (rem == 1u) & (dV == 1u);
    const uint32_t x = s_ctz(bvS | 0x100u) & 7u;
    /* ... and when x is the victim's home itself, it takes the notice (an EVICT_SHARED at the
     * block's home, :498-505) as an eviction from itself: its bit cleared, none left, the entry
     * UNOWNED, its own line untouched */
    const bool selfn = SER_NOTICE_HOME & notice & (x == vh);
    const bool clrM = mod & (dV == 0u) & had;                   /* EVICT_MODIFIED :544-547 */
    const uint32_t nmemV = mod ? Lv : memV;
    const uint32_t nbvV = mod ? (clrM ? 0u : bvV) : (selfn ? 0u : (had ? bvS : bvV));   /* :501-508 */
    const uint32_t ndV = mod ? (clrM ? 2u : dV) : (notice ? (selfn ? 2u : 0u) : ((had & (rem == 0u)) ? 2u : dV));
    const uint32_t mbV2 = (mbV & ~(0xFFFFu << hv)) | ((nmemV | (nbvV << 8)) << hv);
    const uint32_t dsV2 = (dsV & ~(3u << sv)) | (ndV << sv);
    const uint32_t mbH = (ev & (wV == wH)) ? mbV2 : mbH0;
    const uint32_t dsH = (ev & (vh == h)) ? dsV2 : dsH0;
    const uint32_t hh = 16u * (b & 1u), shb = 2u * b;
    const uint32_t memH = (mbH >> hh) & 0xFFu, bvH = (mbH >> (hh + 8u)) & 0xFFu, dH = (dsH >> shb) & 3u;
    const uint32_t owner = s_ctz(bvH | 0x100u);                 /* findOwner :98-105 */
    const uint32_t others = bvH & ~bit;
    /* EM at another owner o on a miss: the home forwards WRITEBACK_INT / WRITEBACK_INV to o
     * (:222-232, :420-431); o, holding the block in M or E, sends FLUSH / FLUSH_INVACK with its
     * value to the home and the requester (:249-265, :451-467), which take it in the round
     * after (:273-296, :475-496).  S with other sharers on a write or an upgrade: REPLY_ID
     * names them and the requester sends each an INV (:350-362), taken in the round after
     * (:366-373). */
    const bool fwd = miss & (dH == 0u) & (owner != n);
    const bool fan = (miss | upg) & (dH == 1u) & (others != 0u) & ((wr != 0u) | upg);
    const uint32_t o = owner & 7u;
    bool oflush = false;
    uint32_t ctO = 0u, vO = 0u;                                 /* o's control word, the value it flushes */
    if (s_any(fwd)) {     /* rare: the owner's line, read only then (a dependent LDS level) */
        const uint32_t laO = m.ld(S_LA + o), lvO = m.ld(S_LV + o);
        const uint32_t c0 = m.ld(S_CT + o);
        ctO = fwd ? c0 : 0u;
        oflush = fwd & (((laO >> sh8) & 0xFFu) == a) & (((c0 >> lsh) & 3u) <= 1u);
        vO = fwd ? (lvO >> sh8) & 0xFFu : 0u;
    }
    /* a forward to an owner that no longer holds the block in M or E: the owner ignores it
     * (:266-270, :468-472), no flush comes and the requester waits for good -- the system's
     * last transaction (every other node waits or has dumped), applied here too: the home's
     * directory and memory as for any forward, the requester's line as the miss left it
     * (INVALID, the address, value 0, :623-625, :675-677), and the system ends */
    const bool dead = fwd & !oflush;
    /* not applied here (ser_step takes them one action at a time): a home >= NP (the defined
     * ASSERT_FAILED), EM with no bit (the reference's assert; never reached, DESIGN), and the
     * rare collisions whose inbox order would differ: the notice to the home or to the
     * victim's home, or to the forward's owner, or to a sharer the fan-out also invalidates */
    const bool ok = ((NP == 8) || (h < (uint32_t)NP)) & (SER_DEAD_FWD | !dead) &
                    !((dH == 0u) & miss & (bvH == 0u)) &
                    !(notice & ((((x == h) | (x == vh)) & !SER_NOTICE_HOME) | (fwd & (x == o)) |
                                (fan & (((others >> x) & 1u) != 0u))));
    if (!ok) return false;
    stamp(2);
    /* the home's directory entry and memory after the request (:188-236, :298-328, :375-435):
     * READ_REQUEST U -> EM {n}, S -> S + n, EM at n unchanged, EM at o -> S {o, n};
     * WRITE_REQUEST writes memory first, then U / S -> EM {n}, EM at n unchanged, EM at o ->
     * EM {n}; UPGRADE -> EM {n}.  A flush then writes o's value to memory (FLUSH_INVACK also
     * EM {n}: unchanged). */
    const bool rdq = miss & (wr == 0u), req = miss | upg;
    const bool keep = miss & (dH == 0u) & !fwd;                 /* EM at the requester */
    const bool excl = !(rdq & (dH == 1u)) & !fwd;               /* REPLY_RD's bitVector == 2 */
    const uint32_t nmemH = (fwd & !dead) ? vO : ((miss & (wr != 0u)) ? val : memH);
    const uint32_t nbvH = rdq ? (dH == 2u ? bit : (((dH == 1u) | fwd) ? (bvH | bit) : bvH)) : (keep ? bvH : bit);
    const uint32_t ndH = rdq ? (dH == 2u ? 0u : (fwd ? 1u : dH)) : 0u;
    /* write-back, branch-free (a disabled store goes to the dummy word); when the eviction's
     * and the request's words coincide the request's write holds both */
    m.st_if(req, S_DS + h, (dsH & ~(3u << shb)) | (ndH << shb));
    m.st_if(req, wH, (mbH & ~(0xFFFFu << hh)) | ((nmemH | (nbvH << 8)) << hh));
    m.st_if(ev & (vh != h), S_DS + vh, dsV2);
    m.st_if(ev & (wV != wH), wV, mbV2);
    /* the forward's owner: S after FLUSH, I after FLUSH_INVACK */
    m.st_if(fwd & !dead, S_CT + o, (ctO & ~(3u << lsh)) | ((wr ? 3u : 2u) << lsh));
    /* the notice's target: its line (same index) S -> E when it still holds the victim */
    if (s_any(notice & !selfn)) {
        const uint32_t laX = m.ld(S_LA + x), ctX = m.ld(S_CT + x);
        const bool up = notice & !selfn & (((laX >> sh8) & 0xFFu) == La) & (((ctX >> lsh) & 3u) == 2u);
        m.st_if(up, S_CT + x, (ctX & ~(3u << lsh)) | (1u << lsh));
    }
    /* the fan-out's sharers: a line holding the block in S or E becomes INVALID */
    uint32_t fs = fan ? others : 0u;
    while (fs) {
        const uint32_t i = s_ctz(fs);
        fs &= fs - 1u;
        const uint32_t laI = m.ld(S_LA + i), ctI = m.ld(S_CT + i), lsI = (ctI >> lsh) & 3u;
        const bool inv = (((laI >> sh8) & 0xFFu) == a) & ((lsI == 1u) | (lsI == 2u));
        m.st_if(inv, S_CT + i, ctI | (3u << lsh));
    }
    /* the requester's line (:243-246, :291-294, :445-447, :334-336, :491-494; a write hit
     * :642-643, :656-657), pendingWriteValue (:633), the instruction index */
    const uint32_t nLv = dead ? 0u : (fwd ? vO : (wr ? val : (miss ? memH : Lv)));
    const uint32_t nLs = dead ? 3u : (wr ? 0u : (miss ? (excl ? 1u : 2u) : Ls));
    const uint32_t nla = (laW & ~(0xFFu << sh8)) | (a << sh8);
    const uint32_t nlv = (lvW & ~(0xFFu << sh8)) | (nLv << sh8);
    ct = (ct & ~(3u << lsh)) | (nLs << lsh);
    ct = (wr ? ((ct & ~0xFFu) | val) : ct) + (1u << SC_IP);
    ct |= dead ? (uint32_t)SC_WAIT : 0u;
    m.st(S_LA + n, nla);
    m.st(S_LV + n, nlv);
    m.st(S_CT + n, ct);
    cc.ct = ct; cc.la = nla; cc.lv = nlv; cc.node = n;
    stamp(3);
    /* rounds: the issue; the request's round (2, or 3 when the eviction queued before it at
     * the same home); a reply the round after -- or the forward's round, then the flush.
     * The INVs after a REPLY_ID are taken in the round after the reply, the round of the
     * node's next action: they touch only their receivers' lines, which that action does
     * not read, so they are applied here and counted, and the round is the next one's.
     * Messages handled: eviction, notice, request, reply or forward + one or two flushes,
     * INVs. */
    const bool lone = hit & !upg;
    const uint32_t treq = (ev & (vh == h)) ? 3u : 2u;
    r.rounds += lone ? 1u : treq + ((fwd & !dead) ? 2u : 1u);
    r.msgs += lone ? 0u : (ev ? 1u : 0u) + (notice ? 1u : 0u) + 2u + ((fwd & !dead) ? (n != h ? 2u : 1u) : 0u) +
                          (fan ? (uint32_t)__builtin_popcount(others) : 0u);
    r.E = 0u;
    /* the dead end: the requester waits, no node can act after the owner's round -- the
     * system is quiescent (the caller ends it when r.A is empty) */
    r.iss = dead ? (r.iss & ~bit) : r.iss;
    r.A = r.iss;
    r.st = (r.dmp == NPM) ? SS_COMPLETED : SS_DEADLOCKED;
    return true;
}

/* word i of node n's canonical 64-byte record (dsm_node_state); flags = wait | dumped << 1 */
template <class M>
DSM_HD uint32_t ser_rec_word(M &m, uint32_t n, uint32_t flags, int i) {
    if (i < 8) {                        /* memory bytes (words 0-3), bitVector bytes (4-7) */
        const uint32_t k = (uint32_t)i & 3u;
        const uint32_t x = m.ld(S_MB + 8u * n + 2u * k), y = m.ld(S_MB + 8u * n + 2u * k + 1u);
        return dt_perm(y, x, i < 4 ? 0x06040200u : 0x07050301u);
    }
    if (i < 12) {                       /* directory states, a byte per block */
        const uint32_t e = m.ld(S_DS + n) >> (8 * (i - 8));
        return (e & 3u) | (((e >> 2) & 3u) << 8) | (((e >> 4) & 3u) << 16) | (((e >> 6) & 3u) << 24);
    }
    if (i == 12) return m.ld(S_LA + n);  /* cache addresses */
    if (i == 13) return m.ld(S_LV + n);  /* cache values    */
    const uint32_t ct = m.ld(S_CT + n);
    if (i == 14) {                      /* cache states, a byte per line */
        const uint32_t e = ct >> SC_LS;
        return (e & 3u) | (((e >> 2) & 3u) << 8) | (((e >> 4) & 3u) << 16) | (((e >> 6) & 3u) << 24);
    }
    return (ct & 0xFFu) | (flags << 8) | ((ct >> SC_IP) << 16);
}

/* record flags of node n at the end: waitingForReply | dumped << 1 */
template <class M>
DSM_HD uint32_t ser_final_flags(M &m, uint32_t n) {
    const uint32_t ct = m.ld(S_CT + n);
    return ((ct & SC_WAIT) ? 1u : 0u) | ((ct & SC_DUMPED) ? 2u : 0u);
}

}  // namespace dsms

#endif
