/*
 * oracle/dsm_oracle.c -- TEST INFRASTRUCTURE ONLY.  Never linked into the product.
 *
 * Clean-room C restatement of the reference's coherence protocol
 * (/root/reference/assignment.c, ruubhagat/HP-Assignment-2) under the deterministic
 * lock-step schedule:
 *   - in round r every node takes exactly one action decided from its state at the start of
 *     the round: (a) pop + handle the inbox head, else (b) idle while waitingForReply, else
 *     (c) issue the next instruction, else (d) dump once, else (e) idle;
 *   - sends are staged and appended to the destination inboxes at the end of the round in
 *     ascending sender id, then program order;
 *   - the system stops after the first round in which no node acted.
 * Each handler cites the reference lines it restates.  Used as the parity checker for the
 * HIP kernels and as bench.py's cpu_baseline ("port").
 */
#include "dsm_oracle.h"
#include <stdio.h>
#include <stdlib.h>
#ifdef _OPENMP
#include <omp.h>
#endif

enum { M_ = 0, E_ = 1, S_ = 2, I_ = 3 };             /* cacheLineState :17 */
enum { DEM = 0, DS = 1, DU = 2 };                    /* directoryEntryState :18 */
enum { READ_REQUEST, WRITE_REQUEST, REPLY_RD, REPLY_WR, REPLY_ID, INV, UPGRADE,
       WRITEBACK_INV, WRITEBACK_INT, FLUSH, FLUSH_INVACK, EVICT_SHARED,
       EVICT_MODIFIED };                             /* transactionType :20-34 */

typedef struct { uint8_t type, sender, addr, value, bv, r2; } omsg;   /* message :53-61 */

typedef struct {
    dsm_rec s;
    uint16_t head, count;
    omsg *ring;
} onode;

typedef struct {
    int np;
    uint32_t cap;
    onode n[8];
    omsg st_msg[256];
    uint8_t st_dest[256];
    int nst;
    int assert_failed;
} osys;

#define WAITING(nd) ((nd)->s.flags & 1)
#define SET_WAITING(nd, v) ((nd)->s.flags = (uint8_t)(((nd)->s.flags & ~1) | ((v) ? 1 : 0)))

static void stage(osys *y, int dest, omsg m) {      /* sendMessage :711-739, staged */
    y->st_dest[y->nst] = (uint8_t)dest;
    y->st_msg[y->nst] = m;
    y->nst++;
}

static int find_owner(const osys *y, uint8_t bv) {   /* findOwner :98-105 */
    for (int i = 0; i < y->np; ++i) if ((bv >> i) & 1) return i;
    return -1;
}
static int count_sharers(const osys *y, uint8_t bv) { /* countSharers :107-115 */
    int c = 0;
    for (int i = 0; i < y->np; ++i) c += (bv >> i) & 1;
    return c;
}

static omsg mk(uint8_t type, int sender, uint8_t addr) {
    omsg m; m.type = type; m.sender = (uint8_t)sender; m.addr = addr; m.value = 0; m.bv = 0;
    m.r2 = 0xFF; return m;
}

/* handleCacheReplacement :742-773 */
static void evict_line(osys *y, int me, int idx) {
    onode *nd = &y->n[me];
    uint8_t a = nd->s.cache_addr[idx], st = nd->s.cache_state[idx];
    if (st == I_ || a == 0xFF) return;                               /* :744-746 */
    omsg m = mk((st == M_) ? EVICT_MODIFIED : EVICT_SHARED, me, a);  /* :759-772 */
    if (st == M_) m.value = nd->s.cache_value[idx];                  /* :767 */
    stage(y, a >> 4, m);
}

/* branch probes for tools/find_scenarios.c (scenario search); compiled out otherwise */
#ifdef ORC_PROBE
void orc_probe(int id);
#define PROBE(id) orc_probe(id)
#else
#define PROBE(id) ((void)0)
#endif

#define OASSERT(c) do { if (!(c)) { PROBE(1000 + __LINE__); y->assert_failed = 1; return; } } while (0)

/* message switch :177-566 */
static void handle(osys *y, int me, omsg m) {
    onode *nd = &y->n[me];
    dsm_rec *s = &nd->s;
    int H = m.addr >> 4, blk = m.addr & 0xF, idx = m.addr % 4;      /* :177-184 */
    int home = (me == H);
    omsg r;
    switch (m.type) {
    case READ_REQUEST:                                               /* :188-236 */
        OASSERT(home);
        r = mk(REPLY_RD, me, m.addr);
        if (s->dir_state[blk] == DU) {                               /* :197-203 */
            s->dir_state[blk] = DEM; s->dir_bv[blk] = (uint8_t)(1u << m.sender);
            r.value = s->memory[blk]; r.bv = 2; stage(y, m.sender, r);
        } else if (s->dir_state[blk] == DS) {                        /* :204-209 */
            s->dir_bv[blk] |= (uint8_t)(1u << m.sender);
            r.value = s->memory[blk]; r.bv = 0; stage(y, m.sender, r);
        } else {                                                     /* :210-234 */
            int o = find_owner(y, s->dir_bv[blk]);
            OASSERT(o != -1);
            if (o == m.sender) {                                     /* :215-221 */
                PROBE(1);
                r.value = s->memory[blk]; r.bv = 2; stage(y, m.sender, r);
            } else {
                omsg f = mk(WRITEBACK_INT, me, m.addr); f.r2 = m.sender;
                stage(y, o, f);
                s->dir_state[blk] = DS; s->dir_bv[blk] |= (uint8_t)(1u << m.sender);
            }
        }
        break;
    case REPLY_RD:                                                   /* :238-247 */
        if (s->cache_addr[idx] != 0xFF && s->cache_addr[idx] != m.addr &&
            s->cache_state[idx] != I_)
            evict_line(y, me, idx);
        s->cache_addr[idx] = m.addr; s->cache_value[idx] = m.value;
        s->cache_state[idx] = (m.bv == 2) ? E_ : S_;
        SET_WAITING(nd, 0);
        break;
    case WRITEBACK_INT:                                              /* :249-271 */
        if (s->cache_addr[idx] == m.addr &&
            (s->cache_state[idx] == M_ || s->cache_state[idx] == E_)) {
            r = mk(FLUSH, me, m.addr); r.value = s->cache_value[idx]; r.r2 = m.r2;
            stage(y, H, r);
            if (m.r2 != H) stage(y, m.r2, r);
            s->cache_state[idx] = S_;
        }                                     /* else ignored (deadlock source) :265-270 */
        break;
    case FLUSH:                                                      /* :273-296 */
        if (home) s->memory[blk] = m.value;                          /* :274-285 */
        if (me == m.r2) {                                            /* :286-295 */
            if (s->cache_addr[idx] != 0xFF && s->cache_addr[idx] != m.addr &&
                s->cache_state[idx] != I_)
                evict_line(y, me, idx);
            s->cache_addr[idx] = m.addr; s->cache_value[idx] = m.value;
            s->cache_state[idx] = S_;
            SET_WAITING(nd, 0);
        }
        break;
    case UPGRADE:                                                    /* :298-328 */
        OASSERT(home);
        if (s->dir_state[blk] == DS) {
            r = mk(REPLY_ID, me, m.addr);
            r.bv = (uint8_t)(s->dir_bv[blk] & ~(1u << m.sender));
            stage(y, m.sender, r);
            s->dir_state[blk] = DEM; s->dir_bv[blk] = (uint8_t)(1u << m.sender);
        } else {                                /* EM or U (:317-326) */
            s->dir_state[blk] = DEM; s->dir_bv[blk] = (uint8_t)(1u << m.sender);
            r = mk(REPLY_ID, me, m.addr); r.bv = 0;
            stage(y, m.sender, r);
        }
        break;
    case REPLY_ID:                                                   /* :330-364 */
        if (s->cache_addr[idx] == m.addr && s->cache_state[idx] != M_) {
            s->cache_value[idx] = s->pending; s->cache_state[idx] = M_;
        } else if (s->cache_addr[idx] == m.addr && s->cache_state[idx] == M_) {
            /* no change :337-338 */
        } else {
            PROBE(3);
            SET_WAITING(nd, 0);                                      /* :345-346 */
            break;
        }
        for (int i = 0; i < y->np; ++i)                              /* :350-362 */
            if (i != me && ((m.bv >> i) & 1)) stage(y, i, mk(INV, me, m.addr));
        SET_WAITING(nd, 0);
        break;
    case INV:                                                        /* :366-373 */
        if (s->cache_addr[idx] == m.addr &&
            (s->cache_state[idx] == S_ || s->cache_state[idx] == E_))
            s->cache_state[idx] = I_;
        break;
    case WRITE_REQUEST:                                              /* :375-435 */
        OASSERT(home);
        s->memory[blk] = m.value;                                    /* :379 */
        if (s->dir_state[blk] == DU) {                               /* :382-391 */
            s->dir_state[blk] = DEM; s->dir_bv[blk] = (uint8_t)(1u << m.sender);
            stage(y, m.sender, mk(REPLY_WR, me, m.addr));
        } else if (s->dir_state[blk] == DS) {                        /* :393-403 */
            r = mk(REPLY_ID, me, m.addr);
            r.bv = (uint8_t)(s->dir_bv[blk] & ~(1u << m.sender));
            stage(y, m.sender, r);
            s->dir_state[blk] = DEM; s->dir_bv[blk] = (uint8_t)(1u << m.sender);
        } else {                                                     /* :405-433 */
            int o = find_owner(y, s->dir_bv[blk]);
            OASSERT(o != -1);
            if (o == m.sender) {                                     /* :410-418 */
                PROBE(2);
                stage(y, m.sender, mk(REPLY_WR, me, m.addr));
            } else {
                omsg f = mk(WRITEBACK_INV, me, m.addr); f.r2 = m.sender;
                stage(y, o, f);
                s->dir_bv[blk] = (uint8_t)(1u << m.sender);           /* :429, stays EM */
            }
        }
        break;
    case REPLY_WR:                                                   /* :437-449 */
        OASSERT(s->cache_addr[idx] == m.addr || s->cache_addr[idx] == 0xFF ||
                s->cache_state[idx] == I_);                          /* :443 */
        s->cache_addr[idx] = m.addr; s->cache_value[idx] = s->pending;
        s->cache_state[idx] = M_;
        SET_WAITING(nd, 0);
        break;
    case WRITEBACK_INV:                                              /* :451-473 */
        if (s->cache_addr[idx] == m.addr &&
            (s->cache_state[idx] == M_ || s->cache_state[idx] == E_)) {
            r = mk(FLUSH_INVACK, me, m.addr); r.value = s->cache_value[idx]; r.r2 = m.r2;
            stage(y, H, r);
            if (m.r2 != H) stage(y, m.r2, r);
            s->cache_state[idx] = I_;
        } else {
            PROBE(4);                             /* ignored (deadlock source) :467-472 */
        }
        break;
    case FLUSH_INVACK:                                               /* :475-496 */
        if (home) {
            s->memory[blk] = m.value;
            s->dir_state[blk] = DEM; s->dir_bv[blk] = (uint8_t)(1u << m.r2);
        }
        if (me == m.r2) {
            OASSERT(s->cache_addr[idx] == m.addr || s->cache_addr[idx] == 0xFF ||
                    s->cache_state[idx] == I_);                      /* :489 */
            s->cache_addr[idx] = m.addr; s->cache_value[idx] = m.value;  /* lost write */
            s->cache_state[idx] = M_;
            SET_WAITING(nd, 0);
        }
        break;
    case EVICT_SHARED:                                               /* :498-539 */
        if (home) {
            if ((s->dir_bv[blk] >> m.sender) & 1) {
                s->dir_bv[blk] &= (uint8_t)~(1u << m.sender);
                int rem = count_sharers(y, s->dir_bv[blk]);
                if (rem == 0) {
                    s->dir_state[blk] = DU;
                } else if (rem == 1 && s->dir_state[blk] == DS) {
                    s->dir_state[blk] = DEM;
                    int o = find_owner(y, s->dir_bv[blk]);
                    if (o != -1) stage(y, o, mk(EVICT_SHARED, me, m.addr));
                }
            }
        } else if (m.sender == H) {                                  /* :526-532 */
            if (s->cache_addr[idx] == m.addr && s->cache_state[idx] == S_)
                s->cache_state[idx] = E_;
        } else {
            PROBE(5);                             /* not from the home: ignored :533-537 */
        }
        break;
    case EVICT_MODIFIED:                                             /* :541-561 */
        OASSERT(home);
        s->memory[blk] = m.value;
        if (s->dir_state[blk] == DEM && ((s->dir_bv[blk] >> m.sender) & 1)) {
            s->dir_bv[blk] = 0; s->dir_state[blk] = DU;
        }
        break;
    default:
        break;
    }
}

/* instruction issue :590-687 (one instruction, already fetched) */
static void issue(osys *y, int me, uint16_t ins) {
    onode *nd = &y->n[me];
    dsm_rec *s = &nd->s;
    int wr = ins >> 15;
    uint8_t a = (uint8_t)((ins >> 8) & 0x7F), v = (uint8_t)(ins & 0xFF);
    int H = a >> 4, idx = a % 4;                                     /* :602-604 */
    if (H >= y->np) { y->assert_failed = 1; return; }               /* out of bounds (:90) */
    int hit = (s->cache_addr[idx] == a && s->cache_state[idx] != I_);
    if (!wr) {                                                       /* :607-630 */
        if (hit) return;
        if (s->cache_addr[idx] != 0xFF && s->cache_state[idx] != I_) evict_line(y, me, idx);
        stage(y, H, mk(READ_REQUEST, me, a));
        SET_WAITING(nd, 1);
        s->cache_state[idx] = I_; s->cache_addr[idx] = a; s->cache_value[idx] = 0;
    } else {                                                         /* :632-685 */
        s->pending = v;                                              /* :633 */
        if (hit) {
            if (s->cache_state[idx] == M_ || s->cache_state[idx] == E_) {   /* :640-645 */
                if (s->cache_state[idx] == E_) PROBE(6);
                s->cache_value[idx] = v; s->cache_state[idx] = M_;
            } else {                                                 /* SHARED :646-659 */
                stage(y, H, mk(UPGRADE, me, a));
                s->cache_value[idx] = v; s->cache_state[idx] = M_;
                SET_WAITING(nd, 1);
            }
        } else {                                                     /* :666-684 */
            if (s->cache_addr[idx] != 0xFF && s->cache_state[idx] != I_)
                evict_line(y, me, idx);
            omsg q = mk(WRITE_REQUEST, me, a); q.value = v;
            stage(y, H, q);
            SET_WAITING(nd, 1);
            s->cache_state[idx] = I_; s->cache_addr[idx] = a; s->cache_value[idx] = 0;
        }
    }
}

/* test hook (tests/model/step_model.cpp): ONE action of node `me` of an np-node system whose
 * node state is *s -- a message {type, sender, addr, value, bv, r2} handled (:177-566), or,
 * with type < 0, the instruction `ins` issued (:590-687).  *s is updated; the staged sends
 * go to out[k] = {dest, type, sender, addr, value, bv, r2}; returns 1 if an assert failed. */
int orc_step(int np, int me, dsm_rec *s, int type, uint16_t ins, int sender, int addr, int value,
             int bv, int r2, uint8_t (*out)[7], int *nout) {
    osys y;
    memset(&y, 0, sizeof y);
    y.np = np; y.cap = DSM_REF_RING_CAP;
    y.n[me].s = *s;
    if (type < 0) {
        issue(&y, me, ins);
    } else {
        omsg m = mk((uint8_t)type, sender, (uint8_t)addr);
        m.value = (uint8_t)value; m.bv = (uint8_t)bv; m.r2 = (uint8_t)r2;
        handle(&y, me, m);
    }
    *s = y.n[me].s;
    for (int k = 0; k < y.nst; ++k) {
        out[k][0] = y.st_dest[k]; out[k][1] = y.st_msg[k].type; out[k][2] = y.st_msg[k].sender;
        out[k][3] = y.st_msg[k].addr; out[k][4] = y.st_msg[k].value; out[k][5] = y.st_msg[k].bv;
        out[k][6] = y.st_msg[k].r2;
    }
    *nout = y.nst;
    return y.assert_failed;
}

static void init_node(dsm_rec *s, int id) {                          /* :778-790, :144-145 */
    for (int i = 0; i < 16; ++i) {
        s->memory[i] = (uint8_t)(20 * id + i);
        s->dir_bv[i] = 0;
        s->dir_state[i] = DU;
    }
    for (int i = 0; i < 4; ++i) {
        s->cache_addr[i] = 0xFF; s->cache_value[i] = 0; s->cache_state[i] = I_;
    }
    s->pending = 0; s->flags = 0; s->issued = 0;
}

typedef struct {
    const uint16_t *trace; uint32_t stride;   /* packed mode */
    int gen; int dist; uint64_t seed; uint64_t sys;  /* generated mode */
} tsrc;

static inline uint16_t fetch(const tsrc *t, int np, int node, uint32_t i) {
    if (t->gen) return dsm_gen_instr(t->seed, t->dist, np, t->sys, node, i);
    return t->trace[(size_t)node * t->stride + i];
}

typedef struct {
    uint64_t seed; uint32_t thresh; uint64_t sys;      /* schedule (dsm_sched_act)         */
    uint32_t *ev; uint32_t ev_cap; uint32_t ev_n;       /* issue order: node << 16 | instr   */
} oextra;

/* round limit of the following runs (orc_set_round_limit; the reference loops forever, the
 * build reports ST_ROUND_LIMIT after this many active rounds) */
static uint32_t g_round_limit = DSM_ROUND_LIMIT;
void orc_set_round_limit(uint32_t limit) { g_round_limit = limit ? limit : DSM_ROUND_LIMIT; }

static int run_one(int np, const tsrc *t, const uint32_t *counts, uint32_t ring_cap,
                   dsm_res *res, dsm_rec *dump_out, dsm_rec *fin_out, uint64_t *by_type,
                   omsg *ring_mem, oextra *x) {
    osys y;
    dsm_rec dump[8];
    memset(&y, 0, sizeof y);
    memset(dump, 0, sizeof dump);
    if (np != 4 && np != 8) return -1;
    if (ring_cap == 0 || ring_cap > DSM_REF_RING_CAP) ring_cap = DSM_REF_RING_CAP;
    y.np = np; y.cap = ring_cap;
    for (int i = 0; i < np; ++i) {
        init_node(&y.n[i].s, i);
        y.n[i].ring = ring_mem + (size_t)i * DSM_REF_RING_CAP;
    }
    uint32_t rounds = 0, msgs = 0, instrs = 0, status = ST_COMPLETED;
    uint64_t bt[DSM_NTYPES] = {0};
    for (uint32_t r = 1;; ++r) {
        int acted = 0;
        y.nst = 0;
        for (int me = 0; me < np; ++me) {
            onode *nd = &y.n[me];
            if (x && x->thresh < DSM_SCHED_LOCKSTEP) {          /* exploration: may stall */
                const int avail = nd->count > 0 ||
                    (!WAITING(nd) && (nd->s.issued < counts[me] || !(nd->s.flags & 2)));
                if (avail && !dsm_sched_act(x->seed, x->thresh, x->sys, r, me)) {
                    acted = 1;
                    continue;
                }
            }
            if (nd->count > 0) {                                     /* drain :158-169 */
                omsg m = nd->ring[nd->head];
                nd->head = (uint16_t)((nd->head + 1) % DSM_REF_RING_CAP);
                nd->count--;
                handle(&y, me, m);
                acted = 1; msgs++; bt[m.type]++;
            } else if (WAITING(nd)) {                                /* :578-581 */
            } else if (nd->s.issued < counts[me]) {                  /* :590-592 */
                uint16_t ins = fetch(t, np, me, nd->s.issued);
                if (x && x->ev) {                              /* DEBUG_INSTR order :596-597 */
                    if (x->ev_n < x->ev_cap) x->ev[x->ev_n] = ((uint32_t)me << 16) | ins;
                    x->ev_n++;
                }
                nd->s.issued++;
                issue(&y, me, ins);
                acted = 1; instrs++;
            } else if (!(nd->s.flags & 2)) {                         /* :688-697 */
                nd->s.flags |= 2;
                dump[me] = nd->s;
                acted = 1;
            }
        }
        if (y.assert_failed) { status = ST_ASSERT_FAILED; rounds = r; break; }
        int ovf = 0;
        for (int k = 0; k < y.nst; ++k) {        /* end-of-round delivery, sender order */
            onode *d = &y.n[y.st_dest[k]];
            if (d->count >= ring_cap) { ovf = 1; break; }
            d->ring[(d->head + d->count) % DSM_REF_RING_CAP] = y.st_msg[k];
            d->count++;
        }
        if (ovf) { status = ST_RING_OVERFLOW; rounds = r; break; }
        if (!acted) {
            int all = 1;
            for (int i = 0; i < np; ++i) all &= (y.n[i].s.flags >> 1) & 1;
            status = all ? ST_COMPLETED : ST_DEADLOCKED;
            break;
        }
        rounds = r;
        if (r >= g_round_limit) { status = ST_ROUND_LIMIT; break; }
    }
    uint32_t mask = 0;
    uint64_t dh = 0, fh = 0;
    for (int i = 0; i < np; ++i) {
        if (y.n[i].s.flags & 2) { mask |= 1u << i; dh += dsm_hash_rec(i, &dump[i], DSM_DUMP_WORDS); }
        fh += dsm_hash_rec(i, &y.n[i].s, DSM_FINAL_WORDS);
        if (dump_out) dump_out[i] = dump[i];
        if (fin_out) fin_out[i] = y.n[i].s;
    }
    res->status = status | (mask << 8);
    res->rounds = rounds; res->msgs = msgs; res->instrs = instrs;
    res->dump_hash = dh; res->final_hash = fh;
    if (by_type) for (int k = 0; k < DSM_NTYPES; ++k) by_type[k] += bt[k];
    return 0;
}

int orc_run_system(int np, const uint16_t *trace, const uint32_t *counts, uint32_t stride,
                   uint32_t ring_cap, dsm_res *res, dsm_rec *dump, dsm_rec *fin,
                   uint64_t *by_type) {
    static __thread omsg *ring_mem;
    if (!ring_mem) ring_mem = (omsg *)malloc(sizeof(omsg) * 8 * DSM_REF_RING_CAP);
    tsrc t; memset(&t, 0, sizeof t); t.trace = trace; t.stride = stride;
    return run_one(np, &t, counts, ring_cap, res, dump, fin, by_type, ring_mem, NULL);
}

int orc_run_packed(int np, const uint16_t *traces, const uint32_t *counts, uint32_t stride,
                   uint64_t n_sys, uint32_t ring_cap, dsm_res *res, dsm_rec *dump,
                   dsm_rec *fin, uint64_t *by_type, int nthreads) {
    uint64_t tot[DSM_NTYPES] = {0};
    int err = 0;
    (void)nthreads;
#pragma omp parallel num_threads(nthreads > 0 ? nthreads : 1) reduction(+:tot[:DSM_NTYPES]) reduction(|:err)
    {
        omsg *ring_mem = (omsg *)malloc(sizeof(omsg) * 8 * DSM_REF_RING_CAP);
#pragma omp for schedule(dynamic, 64)
        for (int64_t i = 0; i < (int64_t)n_sys; ++i) {
            tsrc t; memset(&t, 0, sizeof t);
            t.trace = traces + (size_t)i * np * stride; t.stride = stride;
            err |= run_one(np, &t, counts + (size_t)i * np, ring_cap, &res[i],
                           dump ? dump + (size_t)i * np : NULL, fin ? fin + (size_t)i * np : NULL,
                           tot, ring_mem, NULL);
        }
        free(ring_mem);
    }
    if (by_type) for (int k = 0; k < DSM_NTYPES; ++k) by_type[k] += tot[k];
    return err ? -1 : 0;
}

int orc_run_generated(int np, int dist, uint64_t seed, uint32_t n_instr, uint64_t first_sys,
                      uint64_t n_sys, uint32_t ring_cap, dsm_res *res, uint64_t *by_type,
                      int nthreads) {
    uint64_t tot[DSM_NTYPES] = {0};
    int err = 0;
    (void)nthreads;
#pragma omp parallel num_threads(nthreads > 0 ? nthreads : 1) reduction(+:tot[:DSM_NTYPES]) reduction(|:err)
    {
        omsg *ring_mem = (omsg *)malloc(sizeof(omsg) * 8 * DSM_REF_RING_CAP);
        uint32_t counts[8];
        for (int i = 0; i < 8; ++i) counts[i] = n_instr;
#pragma omp for schedule(dynamic, 256)
        for (int64_t i = 0; i < (int64_t)n_sys; ++i) {
            tsrc t; memset(&t, 0, sizeof t);
            t.gen = 1; t.dist = dist; t.seed = seed; t.sys = first_sys + (uint64_t)i;
            err |= run_one(np, &t, counts, ring_cap, &res[i], NULL, NULL, tot, ring_mem, NULL);
        }
        free(ring_mem);
    }
    if (by_type) for (int k = 0; k < DSM_NTYPES; ++k) by_type[k] += tot[k];
    return err ? -1 : 0;
}

int orc_run_packed_ex(int np, const uint16_t *traces, const uint32_t *counts, uint32_t stride,
                      uint64_t n_sys, uint32_t ring_cap, uint64_t sched_seed,
                      uint32_t sched_thresh, uint64_t first_sys, dsm_res *res, dsm_rec *dump,
                      dsm_rec *fin, uint32_t *issue, uint32_t issue_cap, uint32_t *issue_n,
                      int nthreads) {
    int err = 0;
    (void)nthreads;
#pragma omp parallel num_threads(nthreads > 0 ? nthreads : 1) reduction(|:err)
    {
        omsg *ring_mem = (omsg *)malloc(sizeof(omsg) * 8 * DSM_REF_RING_CAP);
#pragma omp for schedule(dynamic, 64)
        for (int64_t i = 0; i < (int64_t)n_sys; ++i) {
            tsrc t; memset(&t, 0, sizeof t);
            t.trace = traces + (size_t)i * np * stride; t.stride = stride;
            oextra x;
            memset(&x, 0, sizeof x);
            x.seed = sched_seed; x.thresh = sched_thresh; x.sys = first_sys + (uint64_t)i;
            if (issue) { x.ev = issue + (size_t)i * issue_cap; x.ev_cap = issue_cap; }
            err |= run_one(np, &t, counts + (size_t)i * np, ring_cap, &res[i],
                           dump ? dump + (size_t)i * np : NULL, fin ? fin + (size_t)i * np : NULL,
                           NULL, ring_mem, &x);
            if (issue_n) issue_n[i] = x.ev_n;
        }
        free(ring_mem);
    }
    return err ? -1 : 0;
}

void orc_generate(int np, int dist, uint64_t seed, uint32_t n_instr, uint64_t first_sys,
                  uint64_t n_sys, uint16_t *traces, uint32_t *counts) {
    for (uint64_t s = 0; s < n_sys; ++s)
        for (int nd = 0; nd < np; ++nd) {
            if (counts) counts[s * np + nd] = n_instr;
            for (uint32_t i = 0; i < n_instr; ++i)
                traces[(s * np + nd) * n_instr + i] =
                    dsm_gen_instr(seed, dist, np, first_sys + s, nd, i);
        }
}

/* printProcessorState :824-876 restated (byte-exact text, Appendix C of SURVEY.md). */
int orc_format_dump(int node, const dsm_rec *r, char *buf, int cap) {
    static const char *cst[] = {"MODIFIED", "EXCLUSIVE", "SHARED", "INVALID"};
    static const char *dst[] = {"EM", "S", "U"};
    int n = 0;
#define P(...) do { int k = snprintf(buf + n, (size_t)(cap - n), __VA_ARGS__); \
                    if (k < 0 || k >= cap - n) return -1; \
                    n += k; } while (0)
    P("=======================================\n");
    P(" Processor Node: %d\n", node);
    P("=======================================\n\n");
    P("-------- Memory State --------\n");
    P("| Index | Address |   Value  |\n");
    P("|----------------------------|\n");
    for (int i = 0; i < 16; ++i)
        P("|  %3d  |  0x%02X   |  %5d   |\n", i, (node << 4) + i, r->memory[i]);
    P("------------------------------\n\n");
    P("------------ Directory State ---------------\n");
    P("| Index | Address | State |    BitVector   |\n");
    P("|------------------------------------------|\n");
    for (int i = 0; i < 16; ++i)
        P("|  %3d  |  0x%02X   |  %2s   |   0x%08X   |\n", i, (node << 4) + i,
          r->dir_state[i] < 3 ? dst[r->dir_state[i]] : "?", r->dir_bv[i]);
    P("--------------------------------------------\n\n");
    P("------------ Cache State ----------------\n");
    P("| Index | Address | Value |    State    |\n");
    P("|---------------------------------------|\n");
    for (int i = 0; i < 4; ++i)
        P("|  %3d  |  0x%02X   |  %3d  |  %8s \t|\n", i, r->cache_addr[i], r->cache_value[i],
          r->cache_state[i] < 4 ? cst[r->cache_state[i]] : "?");
    P("----------------------------------------\n\n");
#undef P
    return n;
}

uint64_t orc_hash_rec(int node, const dsm_rec *r, int nwords) {
    return dsm_hash_rec(node, r, nwords);
}
