/*
 * tests/model/step_model.cpp -- TEST INFRASTRUCTURE: every row of the transition table
 * (hp-assignment-2_amd/csrc/dsm_table.h, the kernel's datapath) against the oracle's handler
 * (oracle/dsm_oracle.c orc_step), ONE action at a time, on random node states and messages.
 *
 * Whole-system runs (table_model.cpp) only reach the rows a schedule reaches.  Here each
 * message type is delivered to arbitrary states, which also covers rows no trace reaches:
 * REPLY_ID at a line that no longer holds the block (assignment.c:339-346), EVICT_SHARED
 * at a non-home from a node that is not the home (:533-537), the asserts of REPLY_WR /
 * FLUSH_INVACK (:443, :489).  States respect the two invariants dt_compile relies on (a
 * valid line never has address 0xFF; a directory entry in EM holds exactly one bit), and
 * messages reach the nodes the protocol sends them to (home-side types at the home).
 *
 *   step_model <trials> <seed>    -> prints per-row hit counts; exit 1 on the first mismatch
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
#include <tuple>
#include <algorithm>

extern "C" {
#include "dsm_oracle.h"
}
#include "dsm_table.h"

namespace {

uint64_t g_rng;
uint32_t rnd() {
    g_rng = dsm_splitmix(g_rng);
    return (uint32_t)(g_rng >> 32);
}

/* a node state satisfying the kernel's invariants */
void random_state(int np, dsm_rec &s) {
    memset(&s, 0, sizeof s);
    const uint32_t amax = (uint32_t)np * 16u;
    for (int b = 0; b < 16; ++b) {
        s.memory[b] = (uint8_t)rnd();
        const uint32_t st = rnd() % 3;
        s.dir_state[b] = (uint8_t)st;
        if (st == DT_DEM) s.dir_bv[b] = (uint8_t)(1u << (rnd() % np));
        else if (st == DT_DS) { do s.dir_bv[b] = (uint8_t)(rnd() & ((1u << np) - 1u)); while (!s.dir_bv[b]); }
        else s.dir_bv[b] = 0;
    }
    for (int l = 0; l < 4; ++l) {
        const uint32_t st = rnd() % 4;
        s.cache_state[l] = (uint8_t)st;
        /* a line's address has its index bits (a % 4 == l); invalid lines may be 0xFF */
        s.cache_addr[l] = (st == DT_CI && rnd() % 3 == 0) ? 0xFF : (uint8_t)(((rnd() % amax) & ~3u) | (uint32_t)l);
        s.cache_value[l] = (uint8_t)rnd();
    }
    s.pending = (uint8_t)rnd();
    s.flags = (uint8_t)(rnd() & 1u);     /* waitingForReply */
}

struct Msg { int dest, type, sender, addr, value, bv, r2; };

/* fields a receiver reads: the rest are stale in the reference */
std::tuple<int, int, int, int, int, int, int> key(const Msg &m, int np) {
    const int H = m.addr >> 4;
    int v = -1, b = -1, r = -1, x = -1;
    switch (m.type) {
    case DT_WREQ: case DT_EVM: v = m.value; break;
    case DT_RRD: v = m.value; x = (m.bv == 2); break;
    case DT_RID: b = m.bv & ((1 << np) - 1); break;
    case DT_WBINT: case DT_WBINV: r = m.r2; break;
    case DT_FLUSH: case DT_FLINV: v = m.value; r = m.r2; break;
    case DT_EVS: x = m.dest != H ? (m.sender == H) : -1; break;   /* read off the home only */
    default: break;
    }
    return std::make_tuple(m.dest, m.type, m.addr, v, b, r, x);
}

}  // namespace

int main(int argc, char **argv) {
    const long trials = argc > 1 ? atol(argv[1]) : 200000;
    g_rng = argc > 2 ? strtoull(argv[2], 0, 0) : 1;
    static uint32_t tab[DT_TABLE_WORDS];
    if (dt_build(tab) > DT_ENTRIES) { fprintf(stderr, "table too large\n"); return 1; }
    long rows[DT_ENTRIES] = {0};
    long asserts = 0, kinds[20] = {0};
    /* rows no schedule reaches (tools/find_scenarios.c probes: never hit by any trace) */
    long rid_mismatch = 0, evs_not_from_home = 0, rwr_assert = 0, flinv_assert = 0;
    for (long t = 0; t < trials; ++t) {
        const int np = (rnd() & 1) ? 8 : 4;
        const int me = (int)(rnd() % np);
        dsm_rec s;
        random_state(np, s);
        /* the action: a message of a random type delivered where the protocol sends it,
         * or an instruction (RD / WR) */
        const int kind = (int)(rnd() % 15);          /* 0..12 message types, 13-14 issue */
        int type = kind < 13 ? kind : -1;
        int sender = (int)(rnd() % np), r2 = (int)(rnd() % np), value = (int)(rnd() & 0xFF);
        int bv = (int)(rnd() & 0xFF);
        const int blk = (int)(rnd() % 16);
        int H = (int)(rnd() % np);
        bool home_only = type == DT_RREQ || type == DT_WREQ || type == DT_UPG || type == DT_EVM;
        if (home_only) H = me;
        if ((type == DT_FLUSH || type == DT_FLINV) && (rnd() & 1)) r2 = me;
        if ((type == DT_FLUSH || type == DT_FLINV) && H != me) r2 = me;   /* delivered to r2 */
        if (type == DT_EVS && (rnd() & 1)) H = me;                         /* the home part */
        if (type == DT_EVS && H != me && (rnd() & 1)) sender = H;          /* the notify */
        if (type == DT_RRD) bv = (rnd() & 1) ? 2 : 0;
        int addr = (H << 4) | blk;
        /* a reply usually concerns the line the requester holds (as the protocol sends it) */
        if ((type == DT_RRD || type == DT_RWR || type == DT_RID || type == DT_INV ||
             type == DT_WBINT || type == DT_WBINV || type == DT_FLUSH || type == DT_FLINV ||
             type == DT_EVS) && (rnd() % 3) && s.cache_addr[addr & 3] != 0xFF &&
            (int)(s.cache_addr[addr & 3] >> 4) < np && !(home_only))
            addr = s.cache_addr[addr & 3];
        const int wr = kind == 14;
        const uint16_t ins = (uint16_t)((wr << 15) | (addr << 8) | (wr ? value : 0));
        if (type == DT_WBINT || type == DT_WBINV || type == DT_FLUSH || type == DT_FLINV) {
            if ((addr >> 4) != H) H = addr >> 4;
        }

        /* ---- oracle */
        dsm_rec so = s;
        uint8_t out[64][7];
        int nout = 0;
        const int oasrt = orc_step(np, me, &so, type, ins, sender, addr, value, bv, r2, out, &nout);

        /* ---- table datapath (what the kernel computes) */
        DtIn in;
        uint32_t w;
        if (type < 0) {
            w = dt_issue_word(ins);
        } else {
            const uint32_t x = (type == DT_RRD) ? (bv == 2) : (type == DT_EVS) ? (sender == (addr >> 4)) : 0u;
            const uint32_t pay = (type == DT_RID) ? (uint32_t)bv : (uint32_t)value;
            w = (pay & 0xFFu) | ((uint32_t)addr << 8) | (x << 15) | ((uint32_t)type << 16) |
                ((uint32_t)r2 << 20) | ((uint32_t)sender << 24);
        }
        dt_decode(w, &in.a, &in.v, &in.excl, &in.r2, &in.s);
        const uint32_t b = in.a & 15u, idx = in.a & 3u;
        in.op = dt_type(w); in.node = (uint32_t)me; in.np_mask = (1u << np) - 1u;
        in.La = s.cache_addr[idx]; in.Lv = s.cache_value[idx]; in.Ls = s.cache_state[idx];
        in.Db = s.dir_bv[b]; in.Ds = s.dir_state[b]; in.Mv = s.memory[b]; in.pend = s.pending;
        uint32_t evDb;
        const uint32_t opx = dt_opx(in);
        const uint32_t ti = dt_index(in, dt_hdr(tab, opx), &evDb);
        rows[ti]++;
        kinds[kind]++;
        if (type == DT_RID && in.La != in.a) rid_mismatch++;                      /* :339-346 */
        if (type == DT_EVS && (in.a >> 4) != (uint32_t)me && sender != (int)(in.a >> 4))
            evs_not_from_home++;                                                  /* :533-537 */
        const DtOut o = dt_apply(in, tab[2 * ti], tab[2 * ti + 1], evDb);
        dsm_rec st = s;
        st.cache_addr[idx] = (uint8_t)o.nLa; st.cache_value[idx] = (uint8_t)o.nLv;
        st.cache_state[idx] = (uint8_t)o.nLs;
        st.dir_bv[b] = (uint8_t)o.nDb; st.dir_state[b] = (uint8_t)o.nDs; st.memory[b] = (uint8_t)o.nMv;
        if (o.wset) st.flags |= 1;
        if (o.wclr) st.flags &= ~1;
        if (o.pendw) st.pending = (uint8_t)in.v;
        if (type < 0) st.issued = s.issued;        /* the oracle's issue() leaves it too */

        if (oasrt || o.asrt) {
            /* both must assert; the reference aborts, the engine ends the system: the
             * node state and sends of that action are not compared */
            if (!(oasrt && o.asrt)) {
                fprintf(stderr, "trial %ld: assert mismatch (oracle %d, table %d) type %d\n", t, oasrt, (int)o.asrt, type);
                return 1;
            }
            asserts++;
            if (type == DT_RWR) rwr_assert++;                                     /* :443 */
            if (type == DT_FLINV) flinv_assert++;                                 /* :489 */
            continue;
        }
        if (memcmp(&so, &st, sizeof so) != 0) {
            fprintf(stderr, "trial %ld: state mismatch, np %d me %d kind %d addr %02x row %u\n", t, np, me, kind, addr, ti);
            return 1;
        }
        std::vector<std::tuple<int, int, int, int, int, int, int>> a, c;
        for (int k = 0; k < nout; ++k) {
            Msg m{out[k][0], out[k][1], out[k][2], out[k][3], out[k][4], out[k][5], out[k][6]};
            a.push_back(key(m, np));
        }
        for (int wd = 0; wd < 2; ++wd) {
            const uint32_t x = wd ? o.o1 : o.o0;
            for (int d = 0; d < np; ++d)
                if ((x >> (24 + d)) & 1u) {
                    Msg m{d, (int)dt_type(x), me, (int)((x >> 8) & 0x7Fu), (int)(x & 0xFFu),
                          (int)(x & 0xFFu), (int)((x >> 20) & 7u)};
                    if (m.type == DT_RRD) m.bv = ((x >> 15) & 1u) ? 2 : 0;
                    if (m.type == DT_EVS) m.sender = ((x >> 15) & 1u) ? (m.addr >> 4) : -1;
                    c.push_back(key(m, np));
                }
        }
        /* per receiver, in sending order (the only order delivery keeps) */
        std::stable_sort(a.begin(), a.end(), [](auto &p, auto &q) { return std::get<0>(p) < std::get<0>(q); });
        std::stable_sort(c.begin(), c.end(), [](auto &p, auto &q) { return std::get<0>(p) < std::get<0>(q); });
        if (a != c) {
            fprintf(stderr, "trial %ld: sends mismatch, np %d me %d kind %d addr %02x row %u (%zu vs %zu)\n",
                    t, np, me, kind, addr, ti, a.size(), c.size());
            return 1;
        }
    }
    int used = 0;
    for (int r = 0; r < (int)DT_ENTRIES; ++r) used += rows[r] != 0;
    printf("{\"trials\": %ld, \"rows_hit\": %d, \"asserts\": %ld, \"rid_mismatch\": %ld, "
           "\"evs_not_from_home\": %ld, \"rwr_assert\": %ld, \"flinv_assert\": %ld, \"kinds\": [",
           trials, used, asserts, rid_mismatch, evs_not_from_home, rwr_assert, flinv_assert);
    for (int k = 0; k < 15; ++k) printf("%ld%s", kinds[k], k < 14 ? ", " : "]}\n");
    return 0;
}
