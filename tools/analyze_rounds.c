/*
 * tools/analyze_rounds.c -- workload analysis (not product, not a test): runs the oracle's
 * lock-step schedule over generated systems and classifies every round, to size the
 * fast-forward and tail-compaction designs (DESIGN.md "Round anatomy").
 *
 *   gcc -O2 -fopenmp tools/analyze_rounds.c -Ioracle -o /tmp/analyze && /tmp/analyze DIST N [budget]
 *
 * Per round: acting nodes (messages handled / instructions issued / dumps), whether every
 * inbox was empty at the start ("quiet"), and whether the round was a pure hit round (quiet,
 * every acting node issued an instruction that sends nothing: RD hit, WR hit on M/E).
 */
#include "../oracle/dsm_oracle.c"

typedef struct {
    uint64_t rounds, quiet, hitr, segs, acts, acts_msg, acts_ins, hit_ins;
    uint64_t tail_rounds, tail_acts, tail_hitr, tail_segs;
    uint64_t hist[9], tail_hist[9];
    uint64_t single_issuer_quiet;   /* quiet rounds with exactly one issuing node */
} stats;

static int is_hit(const dsm_rec *s, uint16_t ins) {
    int wr = ins >> 15;
    uint8_t a = (uint8_t)((ins >> 8) & 0x7F);
    int idx = a & 3;
    int hit = s->cache_addr[idx] == a && s->cache_state[idx] != I_;
    if (!wr) return hit;
    return hit && (s->cache_state[idx] == M_ || s->cache_state[idx] == E_);
}

static void run_stats(int np, int dist, uint64_t seed, uint32_t n_instr, uint64_t sys,
                      uint32_t budget, stats *st, omsg *ring_mem) {
    osys y;
    memset(&y, 0, sizeof y);
    y.np = np; y.cap = DSM_REF_RING_CAP;
    for (int i = 0; i < np; ++i) { init_node(&y.n[i].s, i); y.n[i].ring = ring_mem + i * DSM_REF_RING_CAP; }
    tsrc t; memset(&t, 0, sizeof t); t.gen = 1; t.dist = dist; t.seed = seed; t.sys = sys;
    int prev_hit = 0;
    for (uint32_t r = 1;; ++r) {
        int quiet = 1, allhit = 1, nact = 0, nmsg = 0, nins = 0;
        for (int me = 0; me < np; ++me) if (y.n[me].count) quiet = 0;
        y.nst = 0;
        for (int me = 0; me < np; ++me) {
            onode *nd = &y.n[me];
            if (nd->count > 0) {
                omsg m = nd->ring[nd->head];
                nd->head = (uint16_t)((nd->head + 1) % DSM_REF_RING_CAP);
                nd->count--;
                handle(&y, me, m);
                nact++; nmsg++; allhit = 0;
            } else if (WAITING(nd)) {
            } else if (nd->s.issued < n_instr) {
                uint16_t ins = fetch(&t, np, me, nd->s.issued);
                if (!is_hit(&nd->s, ins)) allhit = 0; else st->hit_ins++;
                nd->s.issued++;
                issue(&y, me, ins);
                nact++; nins++;
            } else if (!(nd->s.flags & 2)) {
                nd->s.flags |= 2;
                nact++; allhit = 0;
            }
        }
        for (int k = 0; k < y.nst; ++k) {
            onode *d = &y.n[y.st_dest[k]];
            d->ring[(d->head + d->count) % DSM_REF_RING_CAP] = y.st_msg[k];
            d->count++;
        }
        if (!nact || y.assert_failed) break;
        const int hitround = quiet && allhit;
        st->rounds++; st->acts += nact; st->acts_msg += nmsg; st->acts_ins += nins;
        st->hist[nact]++;
        if (quiet) st->quiet++;
        if (quiet && nins == 1 && nmsg == 0) st->single_issuer_quiet++;
        if (hitround) { st->hitr++; if (!prev_hit) st->segs++; }
        if (r > budget) {
            st->tail_rounds++; st->tail_acts += nact; st->tail_hist[nact]++;
            if (hitround) { st->tail_hitr++; if (!prev_hit) st->tail_segs++; }
        }
        prev_hit = hitround;
    }
}

int main(int argc, char **argv) {
    int dist = argc > 1 ? atoi(argv[1]) : 0;
    uint64_t n = argc > 2 ? strtoull(argv[2], 0, 10) : 4096;
    uint32_t budget = argc > 3 ? (uint32_t)atoi(argv[3]) : 4096;
    uint64_t first = argc > 4 ? strtoull(argv[4], 0, 10) : 0;
    stats tot; memset(&tot, 0, sizeof tot);
#pragma omp parallel
    {
        stats st; memset(&st, 0, sizeof st);
        omsg *ring = malloc(sizeof(omsg) * 8 * DSM_REF_RING_CAP);
#pragma omp for schedule(dynamic, 16)
        for (int64_t i = 0; i < (int64_t)n; ++i) run_stats(8, dist, 1, 4096, first + i, budget, &st, ring);
#pragma omp critical
        {
            uint64_t *a = (uint64_t *)&tot, *b = (uint64_t *)&st;
            for (size_t k = 0; k < sizeof st / 8; ++k) a[k] += b[k];
        }
        free(ring);
    }
    printf("dist %d systems %llu\n", dist, (unsigned long long)n);
    printf("rounds/sys %.1f  acts/round %.3f (msg %.3f ins %.3f)  quiet %.3f  hit-rounds %.3f  hit-segments/sys %.1f  hit instrs/sys %.1f\n",
           (double)tot.rounds / n, (double)tot.acts / tot.rounds, (double)tot.acts_msg / tot.rounds,
           (double)tot.acts_ins / tot.rounds, (double)tot.quiet / tot.rounds, (double)tot.hitr / tot.rounds,
           (double)tot.segs / n, (double)tot.hit_ins / n);
    printf("single-issuer quiet rounds %.3f\n", (double)tot.single_issuer_quiet / tot.rounds);
    printf("rounds after non-hit-round compression/sys %.1f\n", (double)(tot.rounds - tot.hitr + tot.segs) / n);
    printf("acting-node histogram:");
    for (int k = 0; k <= 8; ++k) printf(" %d:%.3f", k, (double)tot.hist[k] / tot.rounds);
    printf("\ntail (> %u rounds): rounds/sys %.1f (%.3f of all) acts/round %.3f hit-rounds %.3f segs/sys %.1f\n", budget,
           (double)tot.tail_rounds / n, (double)tot.tail_rounds / tot.rounds,
           tot.tail_rounds ? (double)tot.tail_acts / tot.tail_rounds : 0.0,
           tot.tail_rounds ? (double)tot.tail_hitr / tot.tail_rounds : 0.0, (double)tot.tail_segs / n);
    printf("tail acting-node histogram:");
    for (int k = 0; k <= 8; ++k) printf(" %d:%.3f", k, tot.tail_rounds ? (double)tot.tail_hist[k] / tot.tail_rounds : 0.0);
    printf("\n");
    return 0;
}
