/*
 * tools/analyze_macro.c -- workload analysis (not product, not a test): how much of the serial
 * resume pass's work (the tail, rounds > budget) is one lone node's whole transactions.
 *
 *   gcc -O2 -fopenmp tools/analyze_macro.c -Ioracle -o /tmp/amacro && /tmp/amacro DIST N [budget]
 *
 * The tail is cut at its quiet round starts (no message queued anywhere) into segments.  A
 * segment is a lone-survivor transaction when exactly one node may act at its start (it
 * issues; every other node waits or has dumped) and the segment handles only
 *   the lone node's EVICT_SHARED / EVICT_MODIFIED at the victim's home (no upgrade notice),
 *   its READ_REQUEST / WRITE_REQUEST / UPGRADE at the home, answered to it directly,
 *   the REPLY_RD / REPLY_WR / REPLY_ID that answers it (no INV fan-out);
 * a hit is a one-action segment.  Those are what a transaction macro-step would apply at once.
 */
#include "../oracle/dsm_oracle.c"

typedef struct {
    uint64_t sys_tail, acts, segs;
    uint64_t seg_hit, act_hit;          /* lone hits                           */
    uint64_t seg_tx, act_tx, rnd_tx;    /* lone simple miss transactions       */
    uint64_t seg_lone_other, act_lone_other;
    uint64_t seg_multi, act_multi;      /* several nodes may act at the start  */
    uint64_t seg_dump, act_dump;        /* the lone node's dump                */
    uint64_t tx_len[8];                 /* rounds per simple miss transaction  */
} stats;

static void run_stats(int np, int dist, uint64_t seed, uint32_t n_instr, uint64_t sys,
                      uint32_t budget, stats *st, omsg *ring_mem) {
    osys y;
    memset(&y, 0, sizeof y);
    y.np = np; y.cap = DSM_REF_RING_CAP;
    for (int i = 0; i < np; ++i) { init_node(&y.n[i].s, i); y.n[i].ring = ring_mem + i * DSM_REF_RING_CAP; }
    tsrc t; memset(&t, 0, sizeof t); t.gen = 1; t.dist = dist; t.seed = seed; t.sys = sys;
    /* the open segment */
    int open = 0, lone = -1, simple = 1, acts = 0, rnds = 0, issued = 0, dumped = 0;
    int intail = 0;
    for (uint32_t r = 1;; ++r) {
        int q0 = 0;
        for (int me = 0; me < np; ++me) q0 += y.n[me].count;
        if (r > budget && q0 == 0) {          /* quiet round start: close and open a segment */
            if (open) {
                st->segs++; st->acts += acts;
                if (lone < 0) { st->seg_multi++; st->act_multi += acts; }
                else if (dumped) { st->seg_dump++; st->act_dump += acts; }
                else if (acts == 1 && issued) { st->seg_hit++; st->act_hit++; }
                else if (simple && issued == 1) {
                    st->seg_tx++; st->act_tx += acts; st->rnd_tx += rnds;
                    st->tx_len[rnds < 7 ? rnds : 7]++;
                } else { st->seg_lone_other++; st->act_lone_other += acts; }
            }
            int cand = 0, who = -1;
            for (int me = 0; me < np; ++me) {
                onode *nd = &y.n[me];
                if (!WAITING(nd) && !(nd->s.flags & 2)) { cand++; who = me; }
            }
            open = 1; lone = cand == 1 ? who : -1; simple = 1; acts = 0; rnds = 0; issued = 0;
            dumped = 0; intail = 1;
        }
        y.nst = 0;
        int nact = 0;
        for (int me = 0; me < np; ++me) {
            onode *nd = &y.n[me];
            if (nd->count > 0) {
                omsg m = nd->ring[nd->head];
                nd->head = (uint16_t)((nd->head + 1) % DSM_REF_RING_CAP);
                nd->count--;
                const int before = y.nst;
                handle(&y, me, m);
                nact++;
                if (open && lone >= 0) {
                    const int sent = y.nst - before;
                    int ok;
                    switch (m.type) {
                    case EVICT_SHARED: case EVICT_MODIFIED:
                        ok = m.sender == lone && sent == 0; break;
                    case READ_REQUEST: case WRITE_REQUEST: case UPGRADE:
                        ok = m.sender == lone && sent == 1 && y.st_dest[before] == lone &&
                             y.st_msg[before].type >= REPLY_RD && y.st_msg[before].type <= REPLY_ID;
                        break;
                    case REPLY_RD: case REPLY_WR: case REPLY_ID:
                        ok = me == lone && sent == 0; break;
                    default: ok = 0;
                    }
                    simple &= ok;
                }
            } else if (WAITING(nd)) {
            } else if (nd->s.issued < n_instr) {
                uint16_t ins = fetch(&t, np, me, nd->s.issued);
                nd->s.issued++;
                issue(&y, me, ins);
                nact++;
                if (open) { issued++; simple &= me == lone; }
            } else if (!(nd->s.flags & 2)) {
                nd->s.flags |= 2;
                nact++;
                if (open) dumped = 1;
            }
        }
        if (open) { acts += nact; rnds += nact ? 1 : 0; }
        for (int k = 0; k < y.nst; ++k) {
            onode *d = &y.n[y.st_dest[k]];
            d->ring[(d->head + d->count) % DSM_REF_RING_CAP] = y.st_msg[k];
            d->count++;
        }
        if (!nact || y.assert_failed) break;
    }
    if (intail) st->sys_tail++;
}

int main(int argc, char **argv) {
    int dist = argc > 1 ? atoi(argv[1]) : 0;
    uint64_t n = argc > 2 ? strtoull(argv[2], 0, 10) : 4096;
    uint32_t budget = argc > 3 ? (uint32_t)atoi(argv[3]) : 1024;
    stats tot; memset(&tot, 0, sizeof tot);
#pragma omp parallel
    {
        stats st; memset(&st, 0, sizeof st);
        omsg *ring = malloc(sizeof(omsg) * 8 * DSM_REF_RING_CAP);
#pragma omp for schedule(dynamic, 16)
        for (int64_t i = 0; i < (int64_t)n; ++i) run_stats(8, dist, 1, 4096, (uint64_t)i, budget, &st, ring);
#pragma omp critical
        {
            uint64_t *a = (uint64_t *)&tot, *b = (uint64_t *)&st;
            for (size_t k = 0; k < sizeof st / 8; ++k) a[k] += b[k];
        }
        free(ring);
    }
    const double A = (double)tot.acts;
    printf("dist %d systems %llu budget %u: %llu in the tail, %llu segments, %.0f node-actions\n",
           dist, (unsigned long long)n, budget, (unsigned long long)tot.sys_tail,
           (unsigned long long)tot.segs, A);
    printf("  lone hit          %10llu segs %6.2f%% of actions\n", (unsigned long long)tot.seg_hit, 100 * tot.act_hit / A);
    printf("  lone simple miss  %10llu segs %6.2f%% of actions, %.2f actions %.2f rounds each\n",
           (unsigned long long)tot.seg_tx, 100 * tot.act_tx / A, (double)tot.act_tx / tot.seg_tx,
           (double)tot.rnd_tx / tot.seg_tx);
    printf("  lone other        %10llu segs %6.2f%% of actions, %.2f actions each\n",
           (unsigned long long)tot.seg_lone_other, 100 * tot.act_lone_other / A,
           (double)tot.act_lone_other / (tot.seg_lone_other ? tot.seg_lone_other : 1));
    printf("  lone dump         %10llu segs %6.2f%% of actions\n", (unsigned long long)tot.seg_dump, 100 * tot.act_dump / A);
    printf("  several may act   %10llu segs %6.2f%% of actions, %.2f actions each\n",
           (unsigned long long)tot.seg_multi, 100 * tot.act_multi / A,
           (double)tot.act_multi / (tot.seg_multi ? tot.seg_multi : 1));
    printf("  simple miss rounds:");
    for (int k = 0; k < 8; ++k) if (tot.tx_len[k]) printf(" %d:%.4f", k, (double)tot.tx_len[k] / tot.seg_tx);
    printf("\n");
    return 0;
}
