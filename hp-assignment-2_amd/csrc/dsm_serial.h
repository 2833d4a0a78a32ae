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
 * Inboxes are D-deep FIFOs here (the analysis in DESIGN.md: after round 2^12 a C3 inbox
 * holds at most 2 messages at any moment in 99.9% of systems), continued in a per-node
 * spill FIFO (global memory on the device) when they fill: entries past the first D are
 * appended to the spill and move into the FIFO's tail as its head is popped, so the order is
 * the inbox's.  An inbox that would exceed the inbox limit `cap` (MSG_BUFFER_SIZE, :12, or
 * dsm_set_inbox_limit) ends the system's run here with SR_OVF: the caller hands the system
 * to the 256-deep re-run from scratch, which reports RING_OVERFLOW exactly (the count here
 * can be one higher than at the end of the round, so that hand-off is conservative).
 */
#ifndef DSM_SERIAL_H
#define DSM_SERIAL_H

#include "dsm_table.h"

namespace dsms {

/* per-system words (one LDS column per lane on the device, a plain array on the host):
 *   S_MB + 8n + p   node n, blocks 2p and 2p+1: memory | bitVector << 8 per 16-bit half
 *   S_LN + 4n + i   node n, cache line i: address | value << 8 | state << 16
 *   S_DS + n        node n, directory states (2 bits per block)
 *   S_CT + n        node n, pendingWriteValue | flags << 8 | instructions issued << 16
 *   S_NI + n        node n, instructions in its trace
 *   S_RG + Dn + j   node n, inbox slot j (ring entries: body | sender << 24)
 *   S_RG + 8D       scratch: the target of a disabled (predicated-off) append          */
enum : uint32_t { S_MB = 0, S_LN = 64, S_DS = 96, S_CT = 104, S_NI = 112, S_RG = 120 };
constexpr uint32_t s_words(int D) { return S_RG + 8u * (uint32_t)D + 1u; }   /* + scratch */

/* control bits (the lock-step kernel's C_*): wait 8, dumped 9, assert 11 */
enum : uint32_t { SC_WAIT = DT_CTL_WAIT, SC_DUMPED = 1u << 9, SC_ASSERT = DT_CTL_ASSERT };
enum : uint32_t { SR_RUN = 0, SR_DONE = 1, SR_OVF = 2 };          /* ser_step verdicts */
/* statuses (include/dsm.h DSM_*) */
enum : uint32_t { SS_COMPLETED = 0, SS_DEADLOCKED = 1, SS_ASSERT = 3, SS_ROUND_LIMIT = 4 };
constexpr uint32_t S_LINE_INIT = 0xFFu | (3u << 16);   /* address 0xFF, value 0, INVALID */

/* a system's registers */
struct SReg {
    uint32_t A;       /* nodes still to act in this round                                   */
    uint32_t E;       /* nodes whose inbox was non-empty at the start of this round         */
    uint32_t nz;      /* nodes whose inbox is non-empty now                                 */
    uint32_t iss;     /* nodes neither waiting nor dumped: they issue, or dump, next        */
    uint32_t dmp;     /* nodes that dumped                                                   */
    uint32_t cnt;     /* inbox counts, a nibble per node                                    */
    uint32_t head;    /* inbox heads, a nibble per node                                     */
    uint32_t rounds;  /* active rounds                                                      */
    uint32_t msgs;    /* messages handled                                                   */
    uint32_t asrt;    /* an assert fired in this round                                      */
    uint32_t st;      /* status once SR_DONE                                                */
    uint32_t spl;     /* nodes whose inbox continues in the spill                           */
    uint32_t sc0, sc1;   /* spill counts, a byte per node (nodes 0-3, 4-7)                  */
    uint32_t sh0, sh1;   /* spill heads, a byte per node (a 256-entry ring per node)        */
};

DSM_HD uint32_t s_nib(uint32_t w, uint32_t n) { return (w >> (4u * n)) & 15u; }
DSM_HD uint32_t s_get2(uint32_t w, uint32_t i) { return dt_ubfe(w, 2u * i, 2u); }
DSM_HD uint32_t s_set2(uint32_t w, uint32_t i, uint32_t v) {
    const uint32_t sh = 2u * i;
    return (w & ~(3u << sh)) | (v << sh);
}
DSM_HD uint32_t s_ctz(uint32_t x) { return (uint32_t)__builtin_ctz(x); }
/* byte n of the 8-byte value (hi:lo) -- two registers, not an array (an array indexed at
 * run time goes to scratch memory) */
DSM_HD uint32_t s_byte(uint32_t lo, uint32_t hi, uint32_t n) {
    return (((n & 4u) ? hi : lo) >> (8u * (n & 3u))) & 0xFFu;
}
DSM_HD void s_byte_set(uint32_t &lo, uint32_t &hi, uint32_t n, uint32_t v) {
    const uint32_t sh = 8u * (n & 3u);
    const uint32_t w = (n & 4u) ? hi : lo;
    const uint32_t x = (w & ~(0xFFu << sh)) | (v << sh);
    lo = (n & 4u) ? lo : x;
    hi = (n & 4u) ? x : hi;
}

/* a fresh system: initializeProcessor :778-790 and main :142-146 for every node */
template <int NP, class M>
DSM_HD void ser_fresh(M &m, SReg &r, const uint32_t *counts, uint32_t stride) {
    for (uint32_t n = 0; n < (uint32_t)NP; ++n) {
        for (uint32_t p = 0; p < 8; ++p)
            m.st(S_MB + 8 * n + p, ((20u * n + 2 * p) & 0xFFu) | (((20u * n + 2 * p + 1) & 0xFFu) << 16));
        for (uint32_t i = 0; i < 4; ++i) m.st(S_LN + 4 * n + i, S_LINE_INIT);
        m.st(S_DS + n, 0xAAAAAAAAu);                       /* every block UNOWNED */
        m.st(S_CT + n, 0u);
        m.st(S_NI + n, counts[n] < stride ? counts[n] : stride);
    }
    r.A = r.iss = (1u << NP) - 1u;
    r.E = r.nz = r.dmp = r.cnt = r.head = 0;
    r.rounds = r.msgs = r.asrt = r.st = 0;
    r.spl = r.sc0 = r.sc1 = r.sh0 = r.sh1 = 0;
}

/* one node-action of the system (the lowest node left in this round), then, if it was the
 * round's last, the end of the round.  Branch-free but for the dump record and the rare
 * third-and-later destinations of a multicast: on the device every lane of a wave runs a
 * different system, and divergent branches cost more than the predicated work.
 *   F fetch(node, index, issue) -> the packed instruction (only used when issue);
 *   R on_dump(node): the node's dump record is due (state as stored, flags 2).
 * M: the system's words (ld / st / ld16 / st16) and its spill FIFOs (sp_ld / sp_st (node,
 * index), 256 entries per node).  An append that would make an inbox hold more than cap
 * (<= 256) messages ends the run with SR_OVF.  A disabled append writes the scratch word
 * S_RG + 8D. */
template <int NP, int D, class M, class T, class F, class R>
DSM_HD uint32_t ser_step(M &m, SReg &r, const T &tab, F &&fetch, R &&on_dump, uint32_t lim_rsh,
                         uint32_t cap = 256u) {
    constexpr uint32_t NPM = (1u << NP) - 1u, SCR = S_RG + 8u * (uint32_t)D;
    const uint32_t n = s_ctz(r.A), n4 = 4u * n, bit = 1u << n;
    uint32_t ct = m.ld(S_CT + n);
    const uint32_t nins = m.ld(S_NI + n);
    const uint32_t h0 = s_nib(r.head, n);
    const uint32_t rw = m.ld(S_RG + (uint32_t)D * n + h0);      /* inbox head (may be stale) */
    const bool hasMsg = (r.E & bit) != 0u;                        /* :158-169 */
    const bool doIssue = !hasMsg && (ct >> 16) < nins;            /* :590-592 */
    const bool doDump = !hasMsg && !doIssue;                      /* :688-697 */
    const uint32_t ins = fetch(n, ct >> 16, doIssue);
    const uint32_t w = hasMsg ? rw : dt_issue_word(ins);
    {   /* pop the head */
        const uint32_t hn = (h0 + 1u == (uint32_t)D) ? 0u : h0 + 1u;
        const uint32_t nh = (r.head & ~(15u << n4)) | (hn << n4);
        r.head = hasMsg ? nh : r.head;
        r.cnt -= hasMsg ? (1u << n4) : 0u;
        r.nz &= (hasMsg && s_nib(r.cnt, n) == 0u && !(r.spl & bit)) ? ~bit : ~0u;
        r.msgs += hasMsg ? 1u : 0u;
        if (hasMsg && (r.spl & bit)) {       /* the spill's head moves to the FIFO's tail */
            const uint32_t scn = s_byte(r.sc0, r.sc1, n), shn = s_byte(r.sh0, r.sh1, n);
            uint32_t slot = hn + s_nib(r.cnt, n);
            slot = slot >= (uint32_t)D ? slot - (uint32_t)D : slot;
            m.st(S_RG + (uint32_t)D * n + slot, m.sp_ld(n, shn));
            r.cnt += 1u << n4;
            s_byte_set(r.sh0, r.sh1, n, (shn + 1u) & 0xFFu);
            s_byte_set(r.sc0, r.sc1, n, scn - 1u);
            r.spl &= scn > 1u ? ~0u : ~bit;
        }
    }
    ct += doIssue ? (1u << 16) : 0u;
    const uint32_t op = doDump ? (uint32_t)DT_DUMP : dt_type(w);

    /* decode + micro-op table + datapath (dsm_table.h), as in sim_kernel step (2)-(3) */
    DtIn in;
    dt_decode(w, &in.a, &in.v, &in.excl, &in.r2, &in.s);
    const uint32_t blk = in.a & 15u, idx = in.a & 3u;            /* :177-184 */
    const uint32_t mw = S_MB + 8u * n + (blk >> 1);
    const uint32_t mbw = m.ld16(mw, blk & 1u);
    const uint32_t lw = m.ld(S_LN + 4u * n + idx);
    const uint32_t dsw = m.ld(S_DS + n);
    in.op = op; in.node = n; in.np_mask = NPM;
    in.La = lw & 0xFFu; in.Lv = (lw >> 8) & 0xFFu; in.Ls = lw >> 16;
    in.Db = mbw >> 8; in.Ds = s_get2(dsw, blk); in.Mv = mbw & 0xFFu; in.pend = ct & 0xFFu;
    uint32_t hix = op | ((in.a >> 4) == n ? 32u : 0u);
    if (NP < 8) hix = (op == DT_RD && (in.a >> 4) >= (uint32_t)NP) ? (uint32_t)DT_ASSERT : hix;
    uint32_t evDb;
    const uint32_t ti = dt_index(in, tab.hdr(hix), &evDb);
    uint32_t W0, W1;
    tab.row(ti, W0, W1);
    const uint32_t X = dt_perm(lw, w, 0x05040001u) & ~0x80u;
    const uint32_t Y = dt_perm(mbw, ct, 0x0C050400u) | ((evDb & 0xFFu) << 24);
    const DtOut o = dt_apply_xy(in, X, Y, W0, W1, evDb);
    m.st(S_LN + 4u * n + idx, dt_perm(o.S, o.P, 0x0C040100u));   /* nLa nLv nLs */
    m.st(S_DS + n, s_set2(dsw, blk, o.nDs));
    m.st16(mw, blk & 1u, o.nMv | (o.nDb << 8));
    ct = (ct & ~o.cclr) | o.cset | (doDump ? SC_DUMPED : 0u);   /* wait, pending (:633), assert */
    m.st(S_CT + n, ct);
    r.dmp |= doDump ? bit : 0u;
    if (doDump) on_dump(n);                  /* printProcessorState(threadId, node), :695 */
    r.iss = (ct & (SC_WAIT | SC_DUMPED)) ? (r.iss & ~bit) : (r.iss | bit);
    r.asrt |= ct & SC_ASSERT;

    /* sendMessage :711-739: the first word to its destinations in ascending order, then the
     * second; each to the tail of the receiver's inbox */
    bool ovf = false;
    auto append = [&](bool en, uint32_t d, uint32_t e) {
        const uint32_t c = s_nib(r.cnt, d);
        const bool sp = (r.spl >> d) & 1u;
        const uint32_t scd = sp ? s_byte(r.sc0, r.sc1, d) : 0u;
        const bool over = en && c + scd >= cap;
        const bool fifo = en && !over && !sp && c < (uint32_t)D;
        const bool spill = en && !over && !fifo;
        ovf = ovf || over;
        uint32_t slot = s_nib(r.head, d) + c;
        slot = slot >= (uint32_t)D ? slot - (uint32_t)D : slot;
        m.st(fifo ? S_RG + (uint32_t)D * d + slot : SCR, e);
        r.cnt += fifo ? 1u << (4u * d) : 0u;
        r.nz |= en && !over ? 1u << d : 0u;
        if (spill) {                          /* the FIFO is full: continue in the spill */
            m.sp_st(d, (s_byte(r.sh0, r.sh1, d) + scd) & 0xFFu, e);
            s_byte_set(r.sc0, r.sc1, d, scd + 1u);
            r.spl |= 1u << d;
        }
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
    if (i < 15) {                       /* cache addresses / values / states */
        const uint32_t b = (uint32_t)(i - 12);
        const uint32_t sel = 0x0C0C0400u | (b * 0x00000101u);
        const uint32_t l0 = m.ld(S_LN + 4u * n), l1 = m.ld(S_LN + 4u * n + 1u);
        const uint32_t l2 = m.ld(S_LN + 4u * n + 2u), l3 = m.ld(S_LN + 4u * n + 3u);
        return dt_perm(dt_perm(l3, l2, sel), dt_perm(l1, l0, sel), 0x05040100u);
    }
    const uint32_t ct = m.ld(S_CT + n);
    return (ct & 0xFFu) | (flags << 8) | (ct & 0xFFFF0000u);
}

/* record flags of node n at the end: waitingForReply | dumped << 1 */
template <class M>
DSM_HD uint32_t ser_final_flags(M &m, uint32_t n) {
    const uint32_t ct = m.ld(S_CT + n);
    return ((ct & SC_WAIT) ? 1u : 0u) | ((ct & SC_DUMPED) ? 2u : 0u);
}

}  // namespace dsms

#endif
