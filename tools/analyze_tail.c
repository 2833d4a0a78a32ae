/*
 * tools/analyze_tail.c -- workload analysis (not product, not a test): the state of the
 * systems the serial resume pass continues (rounds > budget), to size its layout.
 *
 *   gcc -O2 -fopenmp tools/analyze_tail.c -Ioracle -o /tmp/atail && /tmp/atail DIST N [budget]
 *
 * Per tail round: messages queued in the whole system at the round start, plus those appended
 * during the round (the most a system-wide queue must hold at once in the serial form, where
 * appends land immediately), nodes acting, and the nodes that ever act in a system's tail.
 */
#include "../oracle/dsm_oracle.c"

#define QH 34
typedef struct {
    uint64_t sys_tail, rounds, acts, msgs, ins;
    uint64_t qhist[QH];          /* queued at round start + appended during the round       */
    uint64_t sysmax[QH];         /* per system: max of the above over its tail               */
    uint64_t live[9];            /* per system: nodes that act in its tail                   */
    uint64_t nodeq[QH];          /* per node per round: its inbox at round start + appended  */
} stats;

static void run_stats(int np, int dist, uint64_t seed, uint32_t n_instr, uint64_t sys,
                      uint32_t budget, stats *st, omsg *ring_mem) {
    osys y;
    memset(&y, 0, sizeof y);
    y.np = np; y.cap = DSM_REF_RING_CAP;
    for (int i = 0; i < np; ++i) { init_node(&y.n[i].s, i); y.n[i].ring = ring_mem + i * DSM_REF_RING_CAP; }
    tsrc t; memset(&t, 0, sizeof t); t.gen = 1; t.dist = dist; t.seed = seed; t.sys = sys;
    int mx = -1;
    uint32_t actmask = 0;
    for (uint32_t r = 1;; ++r) {
        int nact = 0, q0 = 0, cnt0[8];
        for (int me = 0; me < np; ++me) { q0 += y.n[me].count; cnt0[me] = y.n[me].count; }
        y.nst = 0;
        uint32_t am = 0;
        for (int me = 0; me < np; ++me) {
            onode *nd = &y.n[me];
            if (nd->count > 0) {
                omsg m = nd->ring[nd->head];
                nd->head = (uint16_t)((nd->head + 1) % DSM_REF_RING_CAP);
                nd->count--;
                handle(&y, me, m);
                nact++; am |= 1u << me;
                if (r > budget) st->msgs++;
            } else if (WAITING(nd)) {
            } else if (nd->s.issued < n_instr) {
                uint16_t ins = fetch(&t, np, me, nd->s.issued);
                nd->s.issued++;
                issue(&y, me, ins);
                nact++; am |= 1u << me;
                if (r > budget) st->ins++;
            } else if (!(nd->s.flags & 2)) {
                nd->s.flags |= 2;
                nact++; am |= 1u << me;
            }
        }
        int add[8] = {0};
        for (int k = 0; k < y.nst; ++k) {
            onode *d = &y.n[y.st_dest[k]];
            d->ring[(d->head + d->count) % DSM_REF_RING_CAP] = y.st_msg[k];
            d->count++;
            add[y.st_dest[k]]++;
        }
        if (!nact || y.assert_failed) break;
        if (r > budget) {
            int q = q0 + y.nst;
            if (q >= QH) q = QH - 1;
            st->qhist[q]++;
            if (q > mx) mx = q;
            st->rounds++; st->acts += nact;
            actmask |= am;
            for (int me = 0; me < np; ++me) {
                int nq = cnt0[me] + add[me];
                st->nodeq[nq >= QH ? QH - 1 : nq]++;
            }
        }
    }
    if (mx >= 0) {
        st->sys_tail++;
        st->sysmax[mx]++;
        st->live[__builtin_popcount(actmask)]++;
    }
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
    printf("dist %d systems %llu budget %u: %llu in the tail, %.1f tail rounds each, %.3f acts/round (msg %.3f ins %.3f)\n",
           dist, (unsigned long long)n, budget, (unsigned long long)tot.sys_tail,
           (double)tot.rounds / tot.sys_tail, (double)tot.acts / tot.rounds,
           (double)tot.msgs / tot.rounds, (double)tot.ins / tot.rounds);
    printf("system queue (start + appended) per round:");
    for (int k = 0; k < QH; ++k) if (tot.qhist[k]) printf(" %d:%.5f", k, (double)tot.qhist[k] / tot.rounds);
    printf("\nper-system max of it:");
    uint64_t c = 0;
    for (int k = 0; k < QH; ++k) if (tot.sysmax[k]) { c += tot.sysmax[k]; printf(" %d:%.5f", k, (double)c / tot.sys_tail); }
    printf("  (cumulative)\nper-node inbox (start + appended):");
    uint64_t nt = 0; for (int k = 0; k < QH; ++k) nt += tot.nodeq[k];
    for (int k = 0; k < QH; ++k) if (tot.nodeq[k]) printf(" %d:%.6f", k, (double)tot.nodeq[k] / nt);
    printf("\nnodes acting in a system's tail:");
    for (int k = 0; k <= 8; ++k) printf(" %d:%.4f", k, (double)tot.live[k] / tot.sys_tail);
    printf("\n");
    return 0;
}
