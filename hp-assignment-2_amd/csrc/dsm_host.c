/*
 * dsm_host.c -- host side of the drop-in boundary (part of libdsm.so; no GPU involved).
 *
 *   dsm_parse_trace_file / dsm_load_test_dir  replace initializeProcessor's trace reader
 *                                             (assignment.c:792-818)
 *   dsm_format_dump / dsm_write_dump          replace printProcessorState (:824-876),
 *                                             byte-for-byte
 *   dsm_node_hash                             canonical 64-bit hash of a node record
 */
#include "dsm.h"

#include <errno.h>
#include <stdio.h>
#include <string.h>

const char *dsm_strerror(int code) {
    switch (code) {
    case DSM_OK: return "ok";
    case DSM_E_INVAL: return "invalid argument";
    case DSM_E_DEVICE: return "no usable gfx950 device or HIP runtime error";
    case DSM_E_NOMEM: return "out of memory";
    case DSM_E_IO: return "file could not be opened or written";
    case DSM_E_FORMAT: return "trace line is neither 'RD <addr>' nor 'WR <addr> <value>'";
    case DSM_E_STATE: return "operation not valid in the current context state";
    case DSM_E_RANGE: return "address outside the simulated nodes (home >= np)";
    default: return "unknown error";
    }
}

int dsm_abi_version(void) { return DSM_ABI_VERSION; }

/* Same chunking as :802-818: fgets into a 20-byte buffer, the count is checked after the
 * read (so line cap+1 is consumed and dropped), %hhx / %hhu store modulo 256. */
int dsm_parse_trace_file(const char *path, uint16_t *out, uint32_t cap, uint32_t *count) {
    if (!path || !count || (cap && !out)) return DSM_E_INVAL;
    FILE *f = fopen(path, "r");
    if (!f) return DSM_E_IO;
    char line[20];
    uint32_t n = 0;
    int rc = DSM_OK;
    while (fgets(line, sizeof line, f) && n < cap) {
        unsigned char a = 0, v = 0;
        int wr;
        if (line[0] == 'R' && line[1] == 'D') {
            if (sscanf(line, "RD %hhx", &a) != 1) { rc = DSM_E_FORMAT; break; }
            wr = 0; v = 0;                                   /* :807-810 */
        } else if (line[0] == 'W' && line[1] == 'R') {
            if (sscanf(line, "WR %hhx %hhu", &a, &v) != 2) { rc = DSM_E_FORMAT; break; }
            wr = 1;                                          /* :811-815 */
        } else {
            rc = DSM_E_FORMAT;  /* the reference counts this chunk with garbage contents */
            break;
        }
        if (a > 0x7F) { rc = DSM_E_RANGE; break; }
        out[n++] = (uint16_t)((wr << 15) | (a << 8) | v);
    }
    fclose(f);
    *count = n;
    return rc;
}

int dsm_load_test_dir(const char *dir_name, int np, uint32_t cap, uint16_t *traces,
                      uint32_t stride, uint32_t *counts) {
    if (!dir_name || !traces || !counts || (np != 4 && np != 8) || cap > stride)
        return DSM_E_INVAL;
    for (int n = 0; n < np; ++n) {
        char path[256];
        snprintf(path, sizeof path, "tests/%s/core_%d.txt", dir_name, n);   /* :794 */
        int rc = dsm_parse_trace_file(path, traces + (size_t)n * stride, cap, &counts[n]);
        if (rc) return rc;
        for (uint32_t i = 0; i < counts[n]; ++i)
            if (((traces[(size_t)n * stride + i] >> 12) & 0x7) >= (unsigned)np)
                return DSM_E_RANGE;
    }
    return DSM_OK;
}

int dsm_format_dump(int node, const dsm_node_state *st, char *buf, size_t cap) {
    static const char *cst[] = {"MODIFIED", "EXCLUSIVE", "SHARED", "INVALID"};  /* :826 */
    static const char *dst[] = {"EM", "S", "U"};                                /* :828 */
    if (!st || !buf) return DSM_E_INVAL;
    size_t n = 0;
#define EMIT(...)                                                                    \
    do {                                                                             \
        int k_ = snprintf(buf + n, cap - n, __VA_ARGS__);                            \
        if (k_ < 0 || (size_t)k_ >= cap - n) return DSM_E_INVAL;                     \
        n += (size_t)k_;                                                             \
    } while (0)
    EMIT("=======================================\n");
    EMIT(" Processor Node: %d\n", node);
    EMIT("=======================================\n\n");
    EMIT("-------- Memory State --------\n");
    EMIT("| Index | Address |   Value  |\n");
    EMIT("|----------------------------|\n");
    for (int i = 0; i < DSM_MEM_SIZE; i++)
        EMIT("|  %3d  |  0x%02X   |  %5d   |\n", i, (node << 4) + i, st->memory[i]);
    EMIT("------------------------------\n\n");
    EMIT("------------ Directory State ---------------\n");
    EMIT("| Index | Address | State |    BitVector   |\n");
    EMIT("|------------------------------------------|\n");
    for (int i = 0; i < DSM_MEM_SIZE; i++)
        EMIT("|  %3d  |  0x%02X   |  %2s   |   0x%08X   |\n", i, (node << 4) + i,
             st->dir_state[i] < 3 ? dst[st->dir_state[i]] : "??", st->dir_bv[i]);
    EMIT("--------------------------------------------\n\n");
    EMIT("------------ Cache State ----------------\n");
    EMIT("| Index | Address | Value |    State    |\n");
    EMIT("|---------------------------------------|\n");
    for (int i = 0; i < DSM_CACHE_SIZE; i++)
        EMIT("|  %3d  |  0x%02X   |  %3d  |  %8s \t|\n", i, st->cache_addr[i],
             st->cache_value[i], st->cache_state[i] < 4 ? cst[st->cache_state[i]] : "????");
    EMIT("----------------------------------------\n\n");
#undef EMIT
    return (int)n;
}

int dsm_write_dump(int node, const dsm_node_state *st, const char *dir) {
    char buf[4096], path[512];
    int len = dsm_format_dump(node, st, buf, sizeof buf);
    if (len < 0) return len;
    if (dir) snprintf(path, sizeof path, "%s/core_%d_output.txt", dir, node);
    else snprintf(path, sizeof path, "core_%d_output.txt", node);         /* :831 */
    FILE *f = fopen(path, "w");
    if (!f) return DSM_E_IO;
    size_t w = fwrite(buf, 1, (size_t)len, f);
    int rc = fclose(f);
    return (w == (size_t)len && rc == 0) ? DSM_OK : DSM_E_IO;
}

int dsm_format_issue_trace(const uint32_t *events, uint32_t n, char *buf, size_t cap) {
    if ((n && !events) || !buf) return DSM_E_INVAL;
    size_t k = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t e = events[i], ins = e & 0xFFFFu;
        const int w = snprintf(buf + k, cap - k, "Processor %u: instr type=%c, address=0x%02X, value=%u\n",
                               e >> 16, (ins >> 15) ? 'W' : 'R', (ins >> 8) & 0x7Fu, ins & 0xFFu);
        if (w < 0 || (size_t)w >= cap - k) return DSM_E_INVAL;                /* :596-597 */
        k += (size_t)w;
    }
    if (k < cap) buf[k] = 0;
    return (int)k;
}

static uint64_t fmix64(uint64_t z) {
    z ^= z >> 33; z *= 0xff51afd7ed558ccdULL;
    z ^= z >> 33; z *= 0xc4ceb9fe1a85ec53ULL;
    z ^= z >> 33;
    return z;
}

uint64_t dsm_node_hash(int node, const dsm_node_state *st, int nwords) {
    uint32_t w[16];
    memcpy(w, st, sizeof w);
    if (nwords > 16) nwords = 16;
    uint64_t h = 0x9E3779B97F4A7C15ULL * (uint64_t)(node + 1);
    for (int i = 0; i < nwords; ++i) h = fmix64(h ^ ((uint64_t)w[i] | ((uint64_t)i << 32)));
    return h;
}

/* one system's term of the aggregate's result digest: a fmix64 chain over the absolute
 * system id and the six result fields (position-sensitive, so a sum of terms pins every
 * system's result, and shards merge by addition) */
uint64_t dsm_result_digest(uint64_t sys_id, const dsm_sys_result *r) {
    uint64_t h = fmix64(sys_id * 0x9E3779B97F4A7C15ULL + 1u);
    h = fmix64(h ^ ((uint64_t)r->status | ((uint64_t)r->rounds << 32)));
    h = fmix64(h ^ ((uint64_t)r->msgs | ((uint64_t)r->instrs << 32)));
    h = fmix64(h ^ r->dump_hash);
    return fmix64(h ^ r->final_hash);
}

int dsm_aggregate_results(const dsm_sys_result *res, uint64_t n_sys, uint64_t first_sys,
                          dsm_aggregate *agg) {
    if (!agg || (n_sys && !res)) return DSM_E_INVAL;
    memset(agg, 0, sizeof *agg);
    for (uint64_t i = 0; i < n_sys; ++i) {
        const dsm_sys_result *r = &res[i];
        agg->systems++;
        agg->msgs += r->msgs;
        agg->instrs += r->instrs;
        agg->rounds += r->rounds;
        if (r->rounds > agg->max_rounds) agg->max_rounds = r->rounds;
        if ((r->status & 0xFFu) < 5u) agg->by_status[r->status & 0xFFu]++;
        agg->sum_dump_hash += r->dump_hash;
        agg->sum_final_hash += r->final_hash;
        agg->result_digest += dsm_result_digest(first_sys + i, r);
    }
    return DSM_OK;
}
