/*
 * tools/find_scenarios.c -- scenario search (not product, not a test): random small 4-node
 * systems run through the oracle with branch probes compiled in (ORC_PROBE); for each
 * wanted branch the first system that reaches it is shrunk (instructions removed one at a
 * time while the branch is still reached) and printed as a tests/scenarios.py program.
 *
 *   gcc -O2 -DORC_PROBE tools/find_scenarios.c -o /tmp/findsc && /tmp/findsc [tries]
 */
#include "../oracle/dsm_oracle.c"

static uint64_t g_hits;   /* probe ids 1..63 */
static uint64_t g_asserts[4];
void orc_probe(int id) {
    if (id < 64) g_hits |= 1ull << id;
    else g_asserts[0] |= 1;
}

static uint64_t rng = 0x1234567;
static uint32_t rnd(void) { rng = dsm_splitmix(rng); return (uint32_t)(rng >> 32); }

#define NPN 4
#define MAXI 12

static int run(uint16_t tr[NPN][MAXI], uint32_t cn[NPN], dsm_res *res) {
    uint16_t flat[NPN * MAXI];
    for (int n = 0; n < NPN; ++n) for (int i = 0; i < MAXI; ++i) flat[n * MAXI + i] = tr[n][i];
    g_hits = 0; g_asserts[0] = 0;
    orc_run_system(NPN, flat, cn, MAXI, 256, res, NULL, NULL, NULL);
    return 0;
}

static int reaches(uint16_t tr[NPN][MAXI], uint32_t cn[NPN], int id) {
    dsm_res r;
    run(tr, cn, &r);
    if (id == 99) return (r.status & 0xFF) == ST_ASSERT_FAILED;
    return (g_hits >> id) & 1;
}

static void shrink(uint16_t tr[NPN][MAXI], uint32_t cn[NPN], int id) {
    int changed = 1;
    while (changed) {
        changed = 0;
        for (int n = 0; n < NPN; ++n)
            for (int i = 0; i < (int)cn[n]; ++i) {
                uint16_t t2[NPN][MAXI]; uint32_t c2[NPN];
                memcpy(t2, tr, sizeof t2); memcpy(c2, cn, sizeof c2);
                for (int k = i; k + 1 < (int)cn[n]; ++k) t2[n][k] = t2[n][k + 1];
                c2[n]--;
                if (reaches(t2, c2, id)) { memcpy(tr, t2, sizeof t2); memcpy(cn, c2, sizeof c2); changed = 1; }
            }
    }
}

int main(int argc, char **argv) {
    long tries = argc > 1 ? atol(argv[1]) : 2000000;
    const int want[] = {1, 2, 3, 4, 5, 6, 99};
    for (unsigned w = 0; w < sizeof want / sizeof want[0]; ++w) {
        int id = want[w], found = 0;
        for (long t = 0; t < tries && !found; ++t) {
            uint16_t tr[NPN][MAXI]; uint32_t cn[NPN];
            /* few addresses, several homes, colliding cache indices */
            static const uint8_t addrs[] = {0x01, 0x05, 0x11, 0x15, 0x19, 0x21, 0x25, 0x31, 0x35};
            for (int n = 0; n < NPN; ++n) {
                cn[n] = rnd() % (MAXI + 1);
                for (int i = 0; i < MAXI; ++i) {
                    uint32_t x = rnd();
                    uint8_t a = addrs[x % 9];
                    tr[n][i] = (x >> 8) & 1 ? (uint16_t)(0x8000 | (a << 8) | ((x >> 16) & 0xFF)) : (uint16_t)(a << 8);
                }
            }
            if (reaches(tr, cn, id)) {
                shrink(tr, cn, id);
                dsm_res r; run(tr, cn, &r);
                printf("probe %d: status %u rounds %u msgs %u instrs %u\n    tr, cn = build(4, [", id,
                       r.status, r.rounds, r.msgs, r.instrs);
                for (int n = 0; n < NPN; ++n) {
                    printf("[");
                    for (int i = 0; i < (int)cn[n]; ++i) {
                        uint16_t x = tr[n][i];
                        if (x >> 15) printf("(\"WR\", 0x%02X, %u)%s", (x >> 8) & 0x7F, x & 0xFF, i + 1 < (int)cn[n] ? ", " : "");
                        else printf("(\"RD\", 0x%02X)%s", (x >> 8) & 0x7F, i + 1 < (int)cn[n] ? ", " : "");
                    }
                    printf("]%s", n + 1 < NPN ? ", " : "])\n");
                }
                found = 1;
            }
        }
        if (!found) printf("probe %d: not reached in %ld random systems\n", id, tries);
    }
    return 0;
}
