/*
 * tests/model/table_model.cpp -- TEST INFRASTRUCTURE: a CPU model of the gfx950 kernel's
 * round (hp-assignment-2_amd/csrc/dsm_table.h: condition vector -> micro-op table ->
 * datapath), run over generated systems.  tests/test_table_model.py compares its per-system
 * results with the oracle's; this pins the transition table without a GPU.
 *
 *   table_model gen <np> <dist> <seed> <n_instr> <first> <n> <ring_cap> <out.bin>
 *   table_model packed <np> <stride> <n> <traces.u16> <counts.u32> <ring_cap> <out.bin>
 * write n dsm_res records (oracle/dsm_common.h layout).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "dsm_common.h"
#include "dsm_table.h"

namespace {

struct Sys {
    int np;
    uint32_t cap;
    dsm_rec n[8];
    dsm_rec dump[8];
    uint32_t ring[8][256];
    uint32_t head[8], cnt[8];
};

struct Src {
    const uint16_t *trace;      /* packed: [np][stride] of this system, else null */
    const uint32_t *counts;
    uint32_t stride;
    int dist; uint64_t seed; uint32_t n_instr; uint64_t sys;
    uint32_t count(int node) const { return trace ? counts[node] : n_instr; }
    uint16_t at(int np, int node, uint32_t i) const {
        return trace ? trace[(size_t)node * stride + i] : dsm_gen_instr(seed, dist, np, sys, node, i);
    }
};

int run_one(Sys &y, const uint32_t *tab, const Src &src, dsm_res *res) {
    const int np = y.np;
    const uint32_t npm = (1u << np) - 1u;
    for (int i = 0; i < np; ++i) {
        dsm_rec &s = y.n[i];
        memset(&s, 0, sizeof s);
        for (int b = 0; b < 16; ++b) { s.memory[b] = (uint8_t)(20 * i + b); s.dir_state[b] = DT_DU; }
        for (int l = 0; l < 4; ++l) { s.cache_addr[l] = 0xFF; s.cache_state[l] = DT_CI; }
        y.head[i] = y.cnt[i] = 0;
    }
    uint32_t rounds = 0, msgs = 0, instrs = 0, status = ST_COMPLETED;
    for (uint32_t r = 1;; ++r) {
        uint32_t o0[8] = {0}, o1[8] = {0};
        int acted = 0, asrt = 0;
        for (int me = 0; me < np; ++me) {
            dsm_rec &s = y.n[me];
            uint32_t w = 0, op;
            if (y.cnt[me]) {
                w = y.ring[me][y.head[me]];
                y.head[me] = (y.head[me] + 1) % 256;
                y.cnt[me]--;
                op = dt_type(w);
                ++msgs;
            } else if (s.flags & 1) {
                op = DT_IDLE;
            } else if (s.issued < src.count(me)) {
                const uint32_t ins = src.at(np, me, s.issued);
                s.issued++;
                ++instrs;
                w = dt_issue_word(ins);
                op = dt_type(w);
            } else if (!(s.flags & 2)) {
                op = DT_DUMP;
                s.flags |= 2;
                y.dump[me] = s;
            } else {
                op = DT_IDLE;
            }
            if (op != DT_IDLE) acted = 1;
            DtIn in;
            dt_decode(w, &in.a, &in.v, &in.excl, &in.r2, &in.s);
            const uint32_t blk = in.a & 15u, idx = in.a & 3u;
            in.op = op; in.node = (uint32_t)me; in.np_mask = npm;
            in.La = s.cache_addr[idx]; in.Lv = s.cache_value[idx]; in.Ls = s.cache_state[idx];
            in.Db = s.dir_bv[blk]; in.Ds = s.dir_state[blk]; in.Mv = s.memory[blk]; in.pend = s.pending;
            uint32_t evDb;
            const uint32_t opx = dt_opx(in);
            const uint32_t ti = dt_index(in, dt_hdr(tab, opx), &evDb);
            const DtOut o = dt_apply(in, tab[2 * ti], tab[2 * ti + 1], evDb);
            s.cache_addr[idx] = (uint8_t)o.nLa; s.cache_value[idx] = (uint8_t)o.nLv;
            s.cache_state[idx] = (uint8_t)o.nLs;
            if (o.nLs != DT_CI && o.nLa == 0xFFu) {     /* the invariant dt_compile relies on */
                fprintf(stderr, "valid line with address 0xFF\n");
                abort();
            }
            if (o.nDs == DT_DEM && __builtin_popcount(o.nDb & npm) != 1) {   /* and dt_index */
                fprintf(stderr, "directory entry in state EM without exactly one bit\n");
                abort();
            }
            s.dir_bv[blk] = (uint8_t)o.nDb; s.dir_state[blk] = (uint8_t)o.nDs;
            s.memory[blk] = (uint8_t)o.nMv;
            if (o.wset) s.flags |= 1;
            if (o.wclr) s.flags &= ~1;
            if (o.pendw) s.pending = (uint8_t)in.v;
            asrt |= (int)o.asrt;
            o0[me] = o.o0; o1[me] = o.o1;
        }
        if (asrt) { status = ST_ASSERT_FAILED; rounds = r; break; }
        int ovf = 0;
        for (int sd = 0; sd < np && !ovf; ++sd)
            for (int k = 0; k < 2 && !ovf; ++k) {
                const uint32_t x = k ? o1[sd] : o0[sd];
                for (int d = 0; d < np; ++d)
                    if ((x >> (24 + d)) & 1u) {
                        if (y.cnt[d] >= y.cap) { ovf = 1; break; }
                        y.ring[d][(y.head[d] + y.cnt[d]) % 256] = dt_ring_entry(x, (uint32_t)sd);
                        y.cnt[d]++;
                    }
            }
        if (ovf) { status = ST_RING_OVERFLOW; rounds = r; break; }
        if (!acted) {
            int all = 1;
            for (int i = 0; i < np; ++i) all &= (y.n[i].flags >> 1) & 1;
            status = all ? ST_COMPLETED : ST_DEADLOCKED;
            break;
        }
        rounds = r;
        if (r >= DSM_ROUND_LIMIT) { status = ST_ROUND_LIMIT; break; }
    }
    uint32_t mask = 0;
    uint64_t dh = 0, fh = 0;
    for (int i = 0; i < np; ++i) {
        if (y.n[i].flags & 2) { mask |= 1u << i; dh += dsm_hash_rec(i, &y.dump[i], DSM_DUMP_WORDS); }
        fh += dsm_hash_rec(i, &y.n[i], DSM_FINAL_WORDS);
    }
    res->status = status | (mask << 8);
    res->rounds = rounds; res->msgs = msgs; res->instrs = instrs;
    res->dump_hash = dh; res->final_hash = fh;
    return 0;
}

}  // namespace

static uint8_t *slurp(const char *path, size_t *len) {
    FILE *f = fopen(path, "rb");
    if (!f) return nullptr;
    fseek(f, 0, SEEK_END);
    *len = (size_t)ftell(f);
    fseek(f, 0, SEEK_SET);
    uint8_t *b = (uint8_t *)malloc(*len ? *len : 1);
    if (fread(b, 1, *len, f) != *len) { fclose(f); free(b); return nullptr; }
    fclose(f);
    return b;
}

int main(int argc, char **argv) {
    const bool gen = argc == 10 && !strcmp(argv[1], "gen");
    const bool packed = argc == 9 && !strcmp(argv[1], "packed");
    if (!gen && !packed) {
        fprintf(stderr, "usage: table_model gen np dist seed n_instr first n ring out\n"
                        "       table_model packed np stride n traces counts ring out\n");
        return 1;
    }
    static uint32_t tab[DT_TABLE_WORDS];
    if (dt_build(tab) > DT_ENTRIES) {
        fprintf(stderr, "micro-op table rows exceed DT_ENTRIES\n");
        return 1;
    }
    const int np = atoi(argv[2]);
    Sys *y = (Sys *)calloc(1, sizeof(Sys));
    y->np = np;
    uint64_t n;
    const char *out;
    dsm_res *res;
    if (gen) {
        const int dist = atoi(argv[3]);
        const uint64_t seed = strtoull(argv[4], 0, 0), first = strtoull(argv[6], 0, 0);
        const uint32_t n_instr = (uint32_t)strtoul(argv[5], 0, 0);
        n = strtoull(argv[7], 0, 0);
        y->cap = (uint32_t)strtoul(argv[8], 0, 0);
        if (y->cap == 0 || y->cap > 256) y->cap = 256;
        out = argv[9];
        res = (dsm_res *)calloc(n ? n : 1, sizeof(dsm_res));
        for (uint64_t i = 0; i < n; ++i) {
            Src src = {nullptr, nullptr, 0, dist, seed, n_instr, first + i};
            run_one(*y, tab, src, &res[i]);
        }
    } else {
        const uint32_t stride = (uint32_t)strtoul(argv[3], 0, 0);
        n = strtoull(argv[4], 0, 0);
        size_t lt = 0, lc = 0;
        const uint16_t *tr = (const uint16_t *)slurp(argv[5], &lt);
        const uint32_t *cn = (const uint32_t *)slurp(argv[6], &lc);
        if (!tr || !cn || lt < n * np * stride * 2 || lc < n * np * 4) return 1;
        y->cap = (uint32_t)strtoul(argv[7], 0, 0);
        if (y->cap == 0 || y->cap > 256) y->cap = 256;
        out = argv[8];
        res = (dsm_res *)calloc(n ? n : 1, sizeof(dsm_res));
        for (uint64_t i = 0; i < n; ++i) {
            Src src = {tr + i * np * stride, cn + i * np, stride, 0, 0, 0, 0};
            run_one(*y, tab, src, &res[i]);
        }
    }
    FILE *f = fopen(out, "wb");
    if (!f || fwrite(res, sizeof(dsm_res), n, f) != n) return 1;
    fclose(f);
    return 0;
}
