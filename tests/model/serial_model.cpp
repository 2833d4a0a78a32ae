/*
 * tests/model/serial_model.cpp -- TEST INFRASTRUCTURE: the serial form of the lock-step round
 * (hp-assignment-2_amd/csrc/dsm_serial.h, the resume-pass kernel's per-lane engine) run on
 * the host over whole systems from their first round, against the oracle
 * (oracle/dsm_oracle.c): per-system status, rounds, messages, instructions, and the dump and
 * final records of every node (as their hashes).  Systems whose queue outgrows its Q slots
 * (8 in the kernel; fewer here to exercise it) continue in the spill (counted as
 * "spilled"); systems whose inbox would exceed the inbox limit end with SR_OVF (the kernel
 * hands them to the 256-deep re-run, which reports RING_OVERFLOW); they are counted, not
 * compared.
 *
 *   serial_model <np> <dist> <n_sys> <Q> <round_limit_log2 (0 = default)> <instr> [inbox cap]
 *   (dist 3: 8-node uniform addresses on a 4-node system, so instructions whose home is
 *   not simulated raise the defined ASSERT_FAILED deviation)
 *   -> JSON {"systems", "compared", "ovf", "by_status": [...]}; exit 1 on the first mismatch
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

extern "C" {
#include "dsm_oracle.h"
}
#include "dsm_serial.h"

namespace {

struct HostCol {
    uint32_t *p;
    uint32_t *spill;                     /* [S_SPILL] */
    uint32_t ld(uint32_t w) const { return p[w]; }
    void st(uint32_t w, uint32_t v) const { p[w] = v; }
    void st_if(bool en, uint32_t w, uint32_t v) const { if (en) p[w] = v; }
    uint32_t ld8(uint32_t w, uint32_t b) const { return reinterpret_cast<const uint8_t *>(&p[w])[b]; }
    void st8(uint32_t w, uint32_t b, uint32_t v) const { reinterpret_cast<uint8_t *>(&p[w])[b] = (uint8_t)v; }
    uint32_t ld16(uint32_t w, uint32_t h) const { return reinterpret_cast<const uint16_t *>(&p[w])[h]; }
    void st16(uint32_t w, uint32_t h, uint32_t v) const { reinterpret_cast<uint16_t *>(&p[w])[h] = (uint16_t)v; }
    uint32_t sp_ld(uint32_t i) const { return spill[i]; }
    void sp_st(uint32_t i, uint32_t v) const { spill[i] = v; }
};
struct HostTab {
    const uint32_t *t;
    uint32_t hdr(uint32_t i) const { return t[2 * DT_ENTRIES + i]; }
    void row(uint32_t i, uint32_t &w0, uint32_t &w1) const { w0 = t[2 * i]; w1 = t[2 * i + 1]; }
};

void to_rec(HostCol &m, uint32_t n, uint32_t flags, dsm_rec *out) {
    uint32_t w[16];
    for (int i = 0; i < 16; ++i) w[i] = dsms::ser_rec_word(m, n, flags, i);
    static_assert(sizeof(dsm_rec) == 64, "record");
    memcpy(out, w, 64);
}

template <int NP, uint32_t Q>
int run(int dist, uint64_t n_sys, uint32_t lim_log2, uint32_t n_instr, uint32_t cap, bool macro) {
    static uint32_t tab[DT_TABLE_WORDS];
    if (dt_build(tab) > DT_ENTRIES) return 2;
    const HostTab T{tab};
    const uint32_t stride = n_instr;
    std::vector<uint16_t> traces((size_t)n_sys * NP * stride);
    std::vector<uint32_t> counts((size_t)n_sys * NP);
    if (dist == 3) {        /* 8-node address range on a 4-node system: homes >= np assert */
        std::vector<uint16_t> t8((size_t)n_sys * 8 * stride);
        std::vector<uint32_t> c8((size_t)n_sys * 8);
        orc_generate(8, 0, 1, n_instr, 0, n_sys, t8.data(), c8.data());
        for (uint64_t s = 0; s < n_sys; ++s)
            for (int n = 0; n < NP; ++n) {
                memcpy(&traces[(s * NP + n) * stride], &t8[(s * 8 + n) * stride], stride * 2);
                counts[s * NP + n] = c8[s * 8 + n];
            }
    } else {
        orc_generate(NP, dist, 1, n_instr, 0, n_sys, traces.data(), counts.data());
    }
    std::vector<dsm_res> ores(n_sys);
    std::vector<dsm_rec> odump((size_t)n_sys * NP), ofin((size_t)n_sys * NP);
    if (lim_log2) orc_set_round_limit(1u << lim_log2);
    orc_run_packed(NP, traces.data(), counts.data(), stride, n_sys, cap, ores.data(), odump.data(),
                   ofin.data(), nullptr, 8);
    const uint32_t lim = lim_log2 ? lim_log2 : 22;
    uint64_t compared = 0, ovf = 0, by_status[5] = {0, 0, 0, 0, 0};
    std::vector<uint32_t> col(dsms::S_WORDS), spill(dsms::S_SPILL);
    uint64_t spilled = 0, n_macro = 0, n_decl = 0, n_decl_dump = 0;
    for (uint64_t s = 0; s < n_sys; ++s) {
        HostCol m{col.data(), spill.data()};
        dsms::SReg r;
        const uint16_t *tr = traces.data() + s * NP * stride;
        dsms::ser_fresh<NP>(m, r, counts.data() + s * NP, stride);
        dsm_rec dump[8];
        memset(dump, 0, sizeof dump);
        auto fetch = [&](uint32_t n, uint32_t i, bool iss) -> uint32_t { return iss ? tr[(size_t)n * stride + i] : 0u; };
        auto on_dump = [&](uint32_t n) { to_rec(m, n, 2u, &dump[n]); };
        auto fetch_try = [&](uint32_t n, uint32_t i, uint32_t &ins) { ins = tr[(size_t)n * stride + i]; return true; };
        uint32_t v;
        bool sp = false;
        dsms::SCache cc;
        dsms::ser_cache_clear(cc);
        do {
            /* as the kernel: a lone node's whole transaction at once when it applies */
            if (macro && cap >= 256u && dsms::ser_quiet_lone(r, lim)) {
                const uint32_t r0 = r.rounds;
                if (dsms::ser_macro<NP>(m, r, cc, fetch_try, on_dump, [](int) {})) {
                    ++n_macro;
                    if (r.rounds - r0 > dsms::SER_MACRO_MAX_ROUNDS) {     /* the quiet-lone margin */
                        fprintf(stderr, "ser_macro advanced %u rounds (> %u)\n", r.rounds - r0,
                                dsms::SER_MACRO_MAX_ROUNDS);
                        return 3;
                    }
                    v = r.A ? dsms::SR_RUN : dsms::SR_DONE;     /* a dead-end forward ends it */
                    continue;
                }
                const uint32_t n0 = dsms::s_ctz(r.A);
                if ((m.ld(dsms::S_CT + n0) >> dsms::SC_IP) >= dsms::s_ni(r, n0)) ++n_decl_dump;
                else ++n_decl;
            }
            v = cap < 256u ? dsms::ser_step<NP, Q, true>(m, r, T, fetch, on_dump, lim, cap)
                           : dsms::ser_step<NP, Q, false>(m, r, T, fetch, on_dump, lim, cap);
            dsms::ser_cache_clear(cc);
            sp = sp || dsms::s_sq(r.q) != 0u;
        } while (v == dsms::SR_RUN);
        spilled += sp;
        if (v == dsms::SR_OVF) { ++ovf; continue; }
        dsm_res mine;
        mine.status = r.st | (r.dmp << 8);
        mine.rounds = r.rounds;
        mine.msgs = r.msgs;
        uint32_t ins = 0;
        uint64_t dh = 0, fh = 0;
        for (uint32_t n = 0; n < (uint32_t)NP; ++n) {
            ins += m.ld(dsms::S_CT + n) >> dsms::SC_IP;
            dsm_rec f;
            to_rec(m, n, dsms::ser_final_flags(m, n), &f);
            fh += dsm_hash_rec((int)n, &f, DSM_FINAL_WORDS);
            if ((r.dmp >> n) & 1u) dh += dsm_hash_rec((int)n, &dump[n], DSM_DUMP_WORDS);
            if (memcmp(&f, &ofin[s * NP + n], 64) != 0) {
                fprintf(stderr, "sys %llu node %u: final record differs\n", (unsigned long long)s, n);
                return 1;
            }
        }
        mine.instrs = ins;
        mine.dump_hash = dh;
        mine.final_hash = fh;
        const dsm_res &o = ores[s];
        if (mine.status != o.status || mine.rounds != o.rounds || mine.msgs != o.msgs ||
            mine.instrs != o.instrs || mine.dump_hash != o.dump_hash || mine.final_hash != o.final_hash) {
            fprintf(stderr, "sys %llu: serial st %x r %u m %u i %u dh %llx fh %llx | oracle st %x r %u m %u i %u dh %llx fh %llx\n",
                    (unsigned long long)s, mine.status, mine.rounds, mine.msgs, mine.instrs,
                    (unsigned long long)mine.dump_hash, (unsigned long long)mine.final_hash, o.status,
                    o.rounds, o.msgs, o.instrs, (unsigned long long)o.dump_hash,
                    (unsigned long long)o.final_hash);
            return 1;
        }
        ++compared;
        ++by_status[r.st];
    }
    printf("{\"systems\": %llu, \"compared\": %llu, \"ovf\": %llu, \"spilled\": %llu, \"macro\": %llu, \"declined\": %llu, \"declined_dump\": %llu, \"by_status\": [%llu, %llu, %llu, %llu, %llu]}\n",
           (unsigned long long)n_sys, (unsigned long long)compared, (unsigned long long)ovf,
           (unsigned long long)spilled, (unsigned long long)n_macro, (unsigned long long)n_decl, (unsigned long long)n_decl_dump,
           (unsigned long long)by_status[0], (unsigned long long)by_status[1],
           (unsigned long long)by_status[2], (unsigned long long)by_status[3],
           (unsigned long long)by_status[4]);
    return 0;
}

}  // namespace

int main(int argc, char **argv) {
    if (argc < 7) return 2;
    const int np = atoi(argv[1]), dist = atoi(argv[2]), D = atoi(argv[4]);   /* D: queue slots Q */
    const uint64_t n = strtoull(argv[3], nullptr, 10);
    const uint32_t lim = (uint32_t)atoi(argv[5]), ni = (uint32_t)atoi(argv[6]);
    const uint32_t cap = argc > 7 ? (uint32_t)atoi(argv[7]) : 256u;
    const bool macro = argc > 8 ? atoi(argv[8]) != 0 : true;   /* ser_macro on (default) */
    if (np == 8 && D == 8) return run<8, 8>(dist, n, lim, ni, cap, macro);
    if (np == 8 && D == 4) return run<8, 4>(dist, n, lim, ni, cap, macro);
    if (np == 8 && D == 2) return run<8, 2>(dist, n, lim, ni, cap, macro);
    if (np == 8 && D == 1) return run<8, 1>(dist, n, lim, ni, cap, macro);
    if (np == 4 && D == 8) return run<4, 8>(dist, n, lim, ni, cap, macro);
    if (np == 4 && D == 4) return run<4, 4>(dist, n, lim, ni, cap, macro);
    if (np == 4 && D == 2) return run<4, 2>(dist, n, lim, ni, cap, macro);
    if (np == 4 && D == 1) return run<4, 1>(dist, n, lim, ni, cap, macro);
    fprintf(stderr, "serial_model: no build for np %d, Q %d\n", np, D);
    return 2;
}
