/*
 * dsm_parse.h -- one trace chunk of initializeProcessor (assignment.c:802-818), shared by the
 * gfx950 parser kernel (dsm_text.hip) and a host model used by the tests.
 *
 * The reference reads each core file with fgets(line, 20, file): a "chunk" is at most 19
 * bytes and ends after the first '\n'.  A chunk starting "RD" is scanned with
 * sscanf(line, "RD %hhx", ...), one starting "WR" with sscanf(line, "WR %hhx %hhu", ...);
 * every chunk counts as one instruction (:817).  This restates glibc's scanf for exactly
 * those two formats (C locale):
 *   - " " matches any run of isspace() bytes, possibly empty;
 *   - %hhx: optional sign, then optional "0x"/"0X" after a leading '0' (the '0' alone is a
 *     complete number: "0x" followed by no hex digit converts to 0), then hex digits;
 *     %hhu: optional sign, then decimal digits;
 *   - the digits are converted as strtoul does (a leading '-' negates modulo 2^64, a
 *     magnitude >= 2^64 saturates to ULONG_MAX) and stored into an unsigned char (mod 256);
 *   - the scan ends at the chunk end or at a NUL byte.
 * Defined deviations (the reference has undefined behaviour there): a chunk that is neither
 * RD nor WR, or whose conversions do not all succeed, is DSM_E_FORMAT (the reference counts
 * an uninitialised instruction); an address > 0x7F (a home node >= 8) is DSM_E_RANGE.
 */
#ifndef DSM_PARSE_H
#define DSM_PARSE_H

#include <stdint.h>

#ifdef __HIPCC__
#define DSM_PHD __host__ __device__ __forceinline__
#else
#define DSM_PHD static inline
#endif

#define DP_CHUNK 19u   /* sizeof(line) - 1, assignment.c:802 */

DSM_PHD uint32_t dp_space(uint32_t ch) { return ch == ' ' || (ch >= 9u && ch <= 13u); }
/* hex digit value, or 16 */
DSM_PHD uint32_t dp_hex(uint32_t ch) {
    const uint32_t lo = ch | 0x20u;
    return (ch >= '0' && ch <= '9') ? ch - '0' : (lo >= 'a' && lo <= 'f') ? lo - 'a' + 10u : 16u;
}

/* Parse chunk c[0..len) (len <= DP_CHUNK).  Returns 0 and the packed instruction
 * (bit 15 WR, bits 8-14 address, bits 0-7 value), or DSM_E_FORMAT (-5) / DSM_E_RANGE (-7). */
template <typename At>
DSM_PHD int dp_parse_chunk_at(At at, uint32_t *packed) {
    uint32_t wr;
    const uint32_t c0 = at(0), c1 = at(1);
    if (c0 == 'R' && c1 == 'D') wr = 0;                      /* :806 */
    else if (c0 == 'W' && c1 == 'R') wr = 1;                 /* :811 */
    else return -5;
    uint32_t p = 2;
    while (dp_space(at(p))) ++p;
    /* %hhx */
    uint32_t neg = 0, nd = 0, ovf = 0;
    uint64_t acc = 0;
    if (at(p) == '+' || at(p) == '-') { neg = at(p) == '-'; ++p; }
    if (at(p) == '0') {
        nd = 1; ++p;
        if ((at(p) | 0x20u) == 'x') ++p;
    }
    for (;;) {
        const uint32_t d = dp_hex(at(p));
        if (d > 15u) break;
        ovf |= (uint32_t)(acc >> 60) != 0u;
        acc = (acc << 4) | d;
        ++nd; ++p;
    }
    if (!nd) return -5;
    const uint32_t a = ovf ? 0xFFu : (uint32_t)((neg ? 0ull - acc : acc) & 0xFFu);
    uint32_t v = 0;
    if (wr) {
        /* " %hhu" */
        while (dp_space(at(p))) ++p;
        neg = 0; nd = 0; ovf = 0; acc = 0;
        if (at(p) == '+' || at(p) == '-') { neg = at(p) == '-'; ++p; }
        for (;;) {
            const uint32_t ch = at(p);
            if (ch < '0' || ch > '9') break;
            ovf |= acc > (0xFFFFFFFFFFFFFFFFull - 9u) / 10u;
            acc = acc * 10u + (ch - '0');
            ++nd; ++p;
        }
        if (!nd) return -5;
        v = ovf ? 0xFFu : (uint32_t)((neg ? 0ull - acc : acc) & 0xFFu);
    }
    if (a > 0x7Fu) return -7;
    *packed = (wr << 15) | (a << 8) | v;
    return 0;
}

/* chunk in a plain byte array; bytes at or past len read as NUL */
DSM_PHD int dp_parse_chunk(const uint8_t *c, uint32_t len, uint32_t *packed) {
    return dp_parse_chunk_at([=](uint32_t i) -> uint32_t { return i < len ? (uint32_t)c[i] : 0u; },
                             packed);
}

#endif
