/*
 * dsm_text.hip -- gfx950 kernels for the two text boundaries of the reference
 * (ruubhagat/HP-Assignment-2, assignment.c), part of libdsm.so:
 *
 *   parse_kernel initializeProcessor's trace reader (:802-818) for whole ensembles of core
 *                files: fgets(line, 20) chunking + sscanf("RD %hhx") / sscanf("WR %hhx %hhu")
 *                (dsm_parse.h) -> packed u16 traces + counts (HBM-read-bound).
 *   fmt_kernel   printProcessorState (:824-876) for whole ensembles: the 55-line dump of every
 *                selected node record, byte-identical to the reference's fprintf output,
 *                written into fixed DSM_DUMP_SLOT-byte slots (HBM-write-bound).
 *   textlen_kernel / textgen_kernel / scan_kernel
 *                synthetic core files in the shipped tests' text format, from the
 *                counter-based generator (bench and test inputs for parse_kernel).
 *
 * parse_kernel: one wave per file (one-wave workgroups), 2 KB windows (32 B per lane, aligned
 * loads, staged in LDS with a 32-byte halo).  A chunk starts at each line start and every 19
 * bytes into a longer line; every lane finds the chunk starts among its 32 bytes (distance
 * to the line start mod 19, the line start carried across lanes by a wave max-scan), a wave
 * prefix sum gives each chunk its instruction index, and each lane decodes the chunks that
 * start in its bytes from LDS with the canonical-line fast path; chunks it declines are
 * scanned exactly (dsm_parse.h) after that loop.  The first failing chunk (by index) ends the
 * file, as the reference's loop would have misbehaved there.
 *
 * Layout of one dump (Appendix C of SURVEY.md): the memory and directory sections are fixed
 * width (%3d / %02X / %5d / %2s / %08X of byte-sized fields), so only the cache section moves:
 * "%8s" of "EXCLUSIVE" is 9 characters, one more than the other three states.  A workgroup
 * stages FR records' texts in LDS -- copy of the per-node template, then one work item per
 * variable field -- and streams the finished slots out with 16-byte non-temporal stores.
 */
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "dsm.h"
#include "dsm_gen.h"
#include "dsm_internal.h"
#include "dsm_parse.h"

#define DEVI __device__ __forceinline__

namespace {

typedef uint32_t v4u32 __attribute__((ext_vector_type(4)));

/* ---- printProcessorState layout (byte offsets in the base 1954-byte text) ------------- */
constexpr uint32_t SLOT = DSM_DUMP_SLOT, SLOT16 = DSM_DUMP_SLOT / 16;
constexpr uint32_t MEM0 = 193, MEML = 31;     /* "|  %3d  |  0x%02X   |  %5d   |\n"      :846 */
constexpr uint32_t DIR0 = 856, DIRL = 45;     /* "|  %3d  |  0x%02X   |  %2s   |   0x%08X   |\n" :856 */
constexpr uint32_t CAC0 = 1748, CACL = 41;    /* "|  %3d  |  0x%02X   |  %3d  |  %8s \t|\n" :867 */
constexpr uint32_t ITEMS = 16 + 16 + 15;      /* memory, directory, cache-section pieces */

DEVI char hexu(uint32_t d) { return (char)(d < 10 ? '0' + d : 'A' + d - 10); }
/* %3d of 0..255 */
DEVI void dec3(char *p, uint32_t v) {
    p[0] = v >= 100 ? (char)('0' + v / 100) : ' ';
    p[1] = v >= 10 ? (char)('0' + (v / 10) % 10) : ' ';
    p[2] = (char)('0' + v % 10);
}

/* FR records per workgroup iteration, NT threads per workgroup */
template <uint32_t FR, uint32_t NT, bool TLDS>
__global__ void __launch_bounds__(NT) fmt_kernel(const uint8_t *recs, uint64_t rec_stride,
                                                 uint64_t n, int np, const uint4 *tpl,
                                                 v4u32 *out, uint32_t *lens) {
    /* TLDS: the np node-id templates live in LDS for the whole kernel (copied once), so a
     * record's text starts from an LDS-to-LDS copy instead of an L2 read, and the next tile's
     * records are fetched into registers while this tile's slots stream out. */
    __shared__ uint4 s_buf[FR * SLOT16];
    __shared__ uint32_t s_rec[FR][16];
    __shared__ uint4 s_tpl[TLDS ? DSM_MAX_NP * SLOT16 : 1];
    char *const sb = reinterpret_cast<char *>(s_buf);
    const uint32_t tid = threadIdx.x;
    if (TLDS) {
        for (uint32_t i = tid; i < (uint32_t)np * SLOT16; i += NT) s_tpl[i] = tpl[i];
    }
    uint4 rv = make_uint4(0, 0, 0, 0);          /* TLDS: this thread's share of the records */
    auto fetch = [&](uint64_t b) {
        const uint32_t nr = (n - b) < FR ? (uint32_t)(n - b) : FR;
        if (tid < nr * 4)
            rv = *reinterpret_cast<const uint4 *>(recs + (b + (tid >> 2)) * rec_stride + (tid & 3u) * 16);
    };
    if (TLDS && (uint64_t)blockIdx.x * FR < n) fetch((uint64_t)blockIdx.x * FR);
    for (uint64_t base = (uint64_t)blockIdx.x * FR; base < n; base += (uint64_t)gridDim.x * FR) {
        const uint32_t nr = (n - base) < FR ? (uint32_t)(n - base) : FR;
        /* (1) node-id template (static text + node-dependent address column) and records */
        if (TLDS) __syncthreads();                       /* s_tpl ready / last tile stored */
        for (uint32_t i = tid; i < nr * SLOT16; i += NT) {
            const uint32_t r = i / SLOT16, c = i - r * SLOT16;
            const uint32_t t = (uint32_t)((base + r) % (uint64_t)np) * SLOT16 + c;
            s_buf[i] = TLDS ? s_tpl[t] : tpl[t];
        }
        if (tid < nr * 4) {
            const uint32_t r = tid >> 2, q = tid & 3u;
            const uint4 v = TLDS ? rv : *reinterpret_cast<const uint4 *>(recs + (base + r) * rec_stride + q * 16);
            s_rec[r][4 * q + 0] = v.x; s_rec[r][4 * q + 1] = v.y;
            s_rec[r][4 * q + 2] = v.z; s_rec[r][4 * q + 3] = v.w;
        }
        __syncthreads();
        if (TLDS && base + (uint64_t)gridDim.x * FR < n) fetch(base + (uint64_t)gridDim.x * FR);
        /* (2) one work item per variable field group */
        /* items ordered type-major (all memory fields of the tile, then directory, then cache
         * pieces), so a wave's iteration runs one item type: no divergence across types */
        for (uint32_t i = tid; i < FR * ITEMS; i += NT) {
            uint32_t r, f;
            if (i < 16 * FR) { r = i >> 4; f = i & 15u; }
            else if (i < 32 * FR) { r = (i - 16 * FR) >> 4; f = 16 + ((i - 16 * FR) & 15u); }
            else { r = (i - 32 * FR) / 15u; f = 32 + (i - 32 * FR) % 15u; }
            if (r >= nr) continue;
            const uint8_t *rb = reinterpret_cast<const uint8_t *>(s_rec[r]);
            char *t = sb + r * SLOT;
            if (f < 16) {                                        /* node.memory[f], %5d */
                dec3(t + MEM0 + MEML * f + 23, rb[f]);
            } else if (f < 32) {                                 /* directory[f-16] */
                const uint32_t k = f - 16, st = rb[32 + k], bv = rb[16 + k];
                char *l = t + DIR0 + DIRL * k;
                l[21] = st == 0 ? 'E' : st < 3 ? ' ' : '?';      /* %2s of "EM" / "S" / "U" */
                l[22] = st == 0 ? 'M' : st == 1 ? 'S' : st == 2 ? 'U' : '?';
                l[38] = hexu(bv >> 4);                           /* 0x%08X of a byte */
                l[39] = hexu(bv & 15u);
            } else {
                /* cache section (:865-870): 3 items per line + 3 for the trailer.  The
                 * template holds the all-MODIFIED layout; "EXCLUSIVE" is one character longer,
                 * so a line after an EXCLUSIVE one (and the trailer) moves and is rewritten
                 * whole, while an unmoved line only gets its fields. */
                const uint32_t q = f - 32;
                const uint32_t em = (rb[56] == 1) | ((rb[57] == 1) << 1) | ((rb[58] == 1) << 2) | ((rb[59] == 1) << 3);
                if (q < 12) {
                    const uint32_t k = q / 3, part = q - 3 * k;
                    const uint32_t sh = __builtin_popcount(em & ((1u << k) - 1u));
                    const bool moved = sh != 0;
                    char *l = t + CAC0 + CACL * k + sh;
                    if (part == 0) {                          /* "|  %3d  |  0x%02X" */
                        const uint32_t a = rb[48 + k];
                        if (moved) {
                            l[0] = '|'; l[1] = ' '; l[2] = ' '; l[3] = ' '; l[4] = ' ';
                            l[5] = (char)('0' + k); l[6] = ' '; l[7] = ' '; l[8] = '|';
                            l[9] = ' '; l[10] = ' '; l[11] = '0'; l[12] = 'x';
                        }
                        l[13] = hexu(a >> 4); l[14] = hexu(a & 15u);
                    } else if (part == 1) {                   /* "   |  %3d  |  " */
                        if (moved) {
                            l[15] = ' '; l[16] = ' '; l[17] = ' '; l[18] = '|'; l[19] = ' '; l[20] = ' ';
                            l[24] = ' '; l[25] = ' '; l[26] = '|'; l[27] = ' '; l[28] = ' ';
                        }
                        dec3(l + 21, rb[52 + k]);
                    } else {                                  /* "%8s \t|\n" */
                        const uint32_t st = rb[56 + k];
                        const char *s8 = st == 0 ? "MODIFIED" : st == 1 ? "EXCLUSIVE"
                                       : st == 2 ? "  SHARED" : st == 3 ? " INVALID" : "    ????";
                        const uint32_t w = st == 1 ? 9u : 8u;
                        for (uint32_t j = 0; j < w; ++j) l[29 + j] = s8[j];
                        if (moved || st == 1) {
                            char *e = l + 29 + w;
                            e[0] = ' '; e[1] = '\t'; e[2] = '|'; e[3] = '\n';
                        }
                    }
                } else if (em) {                              /* trailer moved: 3 x 14 bytes */
                    char *e = t + CAC0 + 4 * CACL + __builtin_popcount(em);
                    const uint32_t j0 = 14u * (q - 12);
                    for (uint32_t j = j0; j < j0 + 14u; ++j) e[j] = j < 40u ? '-' : '\n';
                }
            }
        }
        if (tid < nr) {
            const uint8_t *rb = reinterpret_cast<const uint8_t *>(s_rec[tid]);
            lens[base + tid] = DSM_DUMP_BASE + (rb[56] == 1) + (rb[57] == 1) + (rb[58] == 1) + (rb[59] == 1);
        }
        __syncthreads();
        /* (3) stream the slots out: contiguous, 16 B per lane, written once */
        v4u32 *dst = out + base * SLOT16;
        for (uint32_t i = tid; i < nr * SLOT16; i += NT) {
            const uint4 x = s_buf[i];
            v4u32 y;
            y.x = x.x; y.y = x.y; y.z = x.z; y.w = x.w;
            __builtin_nontemporal_store(y, dst + i);
        }
        if (!TLDS) __syncthreads();
    }
}


/* ---- trace parser ------------------------------------------------------------------- */
constexpr uint32_t PHALO = 32;      /* halo bytes (a chunk is <= 19) */
#ifndef PARSE_PW
#define PARSE_PW 1          /* one-wave workgroups: 1 / 2 / 4 / 8 measured 9.43 / 9.70 / 9.68 / 9.70 ms */
#endif
constexpr uint32_t PW = PARSE_PW;   /* waves per workgroup */

/* aligned 16-byte load through the global address space (in-order vmcnt, not flat) */
DEVI uint4 ldg16(const uint8_t *p) {
    const v4u32 v = *(const __attribute__((address_space(1))) v4u32 *)p;
    return make_uint4(v.x, v.y, v.z, v.w);
}

/* wave64 inclusive scans on DPP (row_shr 1/2/3/4/8, row_bcast 15/31; no LDS round trips) */
#define DPP(x, ctrl, rm, bm, bc) __builtin_amdgcn_update_dpp(0u, (x), (ctrl), (rm), (bm), (bc))
DEVI uint32_t wave_incl_sum(uint32_t x) {
    uint32_t s = x + DPP(x, 0x111, 0xF, 0xF, true);
    s += DPP(x, 0x112, 0xF, 0xF, true);
    s += DPP(x, 0x113, 0xF, 0xF, true);
    s += DPP(s, 0x114, 0xF, 0xE, false);
    s += DPP(s, 0x118, 0xF, 0xC, false);
    s += DPP(s, 0x142, 0xA, 0xF, false);
    s += DPP(s, 0x143, 0xC, 0xF, false);
    return s;
}
DEVI uint32_t umax(uint32_t a, uint32_t b) { return a > b ? a : b; }
DEVI uint32_t wave_incl_max(uint32_t x) {
    uint32_t s = umax(x, DPP(x, 0x111, 0xF, 0xF, true));
    s = umax(s, DPP(x, 0x112, 0xF, 0xF, true));
    s = umax(s, DPP(x, 0x113, 0xF, 0xF, true));
    s = umax(s, DPP(s, 0x114, 0xF, 0xE, false));
    s = umax(s, DPP(s, 0x118, 0xF, 0xC, false));
    s = umax(s, DPP(s, 0x142, 0xA, 0xF, false));
    s = umax(s, DPP(s, 0x143, 0xC, 0xF, false));
    return s;
}
DEVI uint32_t wave_min(uint32_t x) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_xor(x, o, 64);
        x = t < x ? t : x;
    }
    return x;
}

/* ASCII helpers on one byte */
DEVI uint32_t is_dec(uint32_t c) { return (c - '0') < 10u; }
DEVI uint32_t hexval(uint32_t c) {            /* 0..15, or >= 16 */
    const uint32_t lo = c | 0x20u;
    return is_dec(c) ? c - '0' : ((lo - 'a') < 6u ? lo - 'a' + 10u : 16u);
}

/* Fast path for the canonical lines "RD 0xHH\n" and "WR 0xHH D{1,3}\n" (H hex, D decimal),
 * read from the 12 chunk bytes in c0..c2; every other chunk takes dp_parse_chunk_at.  For
 * those two shapes sscanf's result is exactly the one computed here (dsm_parse.h).
 * Returns 1 and *pk when the chunk has one of the shapes (and lim admits it). */
DEVI uint32_t parse_fast(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t lim, uint32_t *pk) {
    /* branch-free: every condition is a bit, every choice a select */
    const uint32_t b4 = c1 & 0xFFu, b5 = (c1 >> 8) & 0xFFu, b6 = (c1 >> 16) & 0xFFu, b7 = c1 >> 24;
    const uint32_t h1 = hexval(b5), h2 = hexval(b6);
    const uint32_t a = (h1 << 4) | h2;
    const uint32_t hexok = (uint32_t)(b4 == 'x') & (uint32_t)((h1 | h2) < 16u) & (uint32_t)(a <= 0x7Fu);
    const uint32_t rd_ok = (uint32_t)(c0 == 0x30204452u) & hexok & (uint32_t)(b7 == '\n') & (uint32_t)(lim >= 8u);
    const uint32_t b9 = (c2 >> 8) & 0xFFu, b10 = (c2 >> 16) & 0xFFu, b11 = c2 >> 24;
    const uint32_t d8 = (c2 & 0xFFu) - '0', d9 = b9 - '0', d10 = b10 - '0';
    const uint32_t e8 = d8 < 10u, e9 = d9 < 10u, e10 = d10 < 10u;
    const uint32_t n10 = e8 & (uint32_t)(b9 == '\n');
    const uint32_t n11 = e8 & e9 & (uint32_t)(b10 == '\n');
    const uint32_t n12 = e8 & e9 & e10 & (uint32_t)(b11 == '\n');
    const uint32_t v = n10 ? d8 : (n11 ? d8 * 10u + d9 : d8 * 100u + d9 * 10u + d10);
    const uint32_t n = n10 ? 10u : (n11 ? 11u : 12u);
    const uint32_t wr_ok = (uint32_t)(c0 == 0x30205257u) & hexok & (uint32_t)(b7 == ' ') &
                           (n10 | n11 | n12) & (uint32_t)(lim >= n);
    *pk = rd_ok ? (a << 8) : ((1u << 15) | (a << 8) | (v & 0xFFu));
    return rd_ok | wr_ok;
}

/* parse_fast's decision and result in word-parallel (SWAR) form: the constant bytes of c1 in
 * one masked compare (b5 in '0'..'7' is the address's high digit under a <= 0x7F), and the
 * WR value's digits and newline as byte masks of c2 (the first non-digit byte must be the
 * newline, at byte 1..3); fewer compare -> lane-mask -> select hops than parse_fast. */
DEVI uint32_t parse_fast_swar(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t lim, uint32_t *pk) {
    const uint32_t rd = (uint32_t)(c0 == 0x30204452u), wr = (uint32_t)(c0 == 0x30205257u);
    const uint32_t want = rd ? 0x0A003078u : 0x20003078u;          /* 'x' '0'..'7' . '\n' | ' ' */
    const uint32_t c1ok = (uint32_t)(((c1 ^ want) & 0xFF00F8FFu) == 0u);
    const uint32_t b6 = (c1 >> 16) & 0xFFu;
    const uint32_t dd = b6 - 0x30u, ll = (b6 | 0x20u) - 0x61u;     /* digit / letter, either case */
    const uint32_t h2ok = (uint32_t)(dd < 10u) | (uint32_t)(ll < 6u);
    const uint32_t a = (((c1 >> 8) & 7u) << 4) | (dd < 10u ? dd : ll + 10u);
    const uint32_t y = c2 ^ 0x30303030u;                            /* digits -> 0..9 */
    const uint32_t nd = (((y & 0x7F7F7F7Fu) + 0x76767676u) | y) & 0x80808080u;  /* non-digit */
    const uint32_t z = c2 ^ 0x0A0A0A0Au;
    const uint32_t nlb = ~((((z & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | z)) & 0x80808080u; /* newline */
    const uint32_t wv = (uint32_t)((nd & (0u - nd) & nlb) != 0u) & (uint32_t)((nd & 0x80u) == 0u);
    const uint32_t p = (uint32_t)__builtin_ctz(nd | 0x80000000u) >> 3;   /* digits before it */
    const uint32_t yy = y << (24u - 8u * p);
    const uint32_t v = (yy & 0xFFu) * 100u + ((yy >> 8) & 0xFFu) * 10u + ((yy >> 16) & 0xFFu);
    *pk = rd ? (a << 8) : ((1u << 15) | (a << 8) | (v & 0xFFu));
    const uint32_t lok = rd ? (uint32_t)(lim >= 8u) : (wr & wv & (uint32_t)(lim >= 9u + p));
    return c1ok & h2ok & lok;
}
/* v_dot4_u32_u8 (a's four bytes times b's, summed, plus c); host form for the decoder tests */
DEVI uint32_t udot4(uint32_t a, uint32_t b, uint32_t c) {
#ifdef __HIP_DEVICE_COMPILE__
    return __builtin_amdgcn_udot4(a, b, c, false);
#else
    for (int i = 0; i < 32; i += 8) c += ((a >> i) & 0xFFu) * ((b >> i) & 0xFFu);
    return c;
#endif
}
/* parse_fast_swar with nothing the compiler turns into a branch: the WR value is one
 * v_dot4_u32_u8 of its digits (aligned to bytes 0-2) with (100, 10, 1), computed for every
 * chunk (a lane's RD and WR chunks are one data flow, not two exec-masked paths), and the
 * address's low digit is (b & 15) + 9 * bit 6 of b once b is known to be a hex digit. */
DEVI uint32_t parse_fast_v3(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t lim, uint32_t *pk) {
    const uint32_t rd = (uint32_t)(c0 == 0x30204452u), wr = (uint32_t)(c0 == 0x30205257u);
    const uint32_t want = 0x0A003078u ^ ((0u - wr) & 0x2A000000u);  /* b7 '\n' (RD) or ' ' (WR) */
    const uint32_t c1ok = (uint32_t)(((c1 ^ want) & 0xFF00F8FFu) == 0u);
    const uint32_t b6 = __builtin_amdgcn_ubfe(c1, 16, 8);
    const uint32_t h2ok = (uint32_t)(b6 - 0x30u < 10u) | (uint32_t)((b6 | 0x20u) - 0x61u < 6u);
    const uint32_t lo4 = (b6 & 15u) + 9u * ((b6 >> 6) & 1u);
    const uint32_t a = (__builtin_amdgcn_ubfe(c1, 8, 3) << 4) | lo4;
    const uint32_t y = c2 ^ 0x30303030u;                            /* digits -> 0..9 */
    const uint32_t nd = (((y & 0x7F7F7F7Fu) + 0x76767676u) | y) & 0x80808080u;  /* non-digit */
    const uint32_t z = c2 ^ 0x0A0A0A0Au;
    const uint32_t nlb = ~((((z & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | z)) & 0x80808080u; /* newline */
    const uint32_t fb = nd & (0u - nd);                             /* first non-digit byte's bit */
    const uint32_t wv = (uint32_t)((fb & nlb) != 0u) & (uint32_t)(fb != 0x80u);
    const uint32_t p = (uint32_t)__builtin_ctz(nd | 0x80000000u) >> 3;   /* digits before it */
    const uint32_t v = udot4(y << (24u - 8u * p), 0x00010A64u, 0u);
    *pk = (wr << 15) | (a << 8) | ((0u - wr) & v & 0xFFu);
    const uint32_t need = wr ? 9u + p : 8u;
    const uint32_t lok = (uint32_t)(lim >= need) & (rd | (wr & wv));
    return c1ok & h2ok & lok;
}
#ifndef PARSE_SWAR
#define PARSE_SWAR 2        /* 2: parse_fast_v3; 1: parse_fast_swar (8.96-8.98 vs 9.31-9.35 ms, parse_fast) */
#endif
#if PARSE_SWAR == 2
#define PARSE_FAST parse_fast_v3
#elif PARSE_SWAR
#define PARSE_FAST parse_fast_swar
#else
#define PARSE_FAST parse_fast
#endif

/* low n bits (n <= 32) */
DEVI uint32_t lowmask(uint32_t n) { return n >= 32u ? 0xFFFFFFFFu : (1u << n) - 1u; }

/* One file per wave; windows of 64 x BPL bytes, double-buffered in registers (the next
 * window's loads are in flight while this one is scanned), staged in LDS for the chunk
 * reads.
 *
 * Two builds of the same kernel.  FAST (the first pass over every file) has no cold path: a
 * window with a line that needs chunks every 19 bytes, or a chunk the canonical-line decoder
 * declines, abandons the whole file, which goes on a device list; the EXACT build (the second
 * pass) reads only the listed files, with the per-byte chunking of long lines and the exact
 * scanner of dsm_parse.h.  Generated and shipped core files never reach the second pass.
 * Splitting them (round 5) took the cold paths' code and registers out of the hot kernel:
 * 77 VGPRs with no spills at 6 waves per SIMD instead of 80 with 8-10 spilled, 7.4 vs 8.4 ms
 * on the bench's 21-GB text. */
#ifndef PARSE_OCC
#define PARSE_OCC 6
#endif
#ifndef PARSE_TRANSPOSE
#define PARSE_TRANSPOSE 1   /* newline mask by one 4 x 8 bit transpose: 8.23-8.36 vs 8.91-8.96 ms */
#endif
#ifndef PARSE_UNI
#define PARSE_UNI 1         /* wave index, and so the file loop, uniform (readfirstlane) */
#endif
#ifndef PARSE_PROBE
#define PARSE_PROBE 0       /* timing probes of the FAST pass (results invalid): 1 no decode, 2 decode
                               without the store, 3 decode with the chunk words from registers */
#endif
template <uint32_t BPL, bool FAST>
__global__ void __launch_bounds__(64 * PW) __attribute__((amdgpu_waves_per_eu(PARSE_OCC)))
parse_kernel(const uint8_t *text, const uint64_t *off, uint64_t n_files, uint32_t cap,
             uint32_t stride, int np, uint16_t *traces, uint32_t *counts, int32_t *status,
             uint32_t *flist, uint32_t *fcount) {
    constexpr uint32_t K = BPL / 16, WIN = 64 * BPL;
    __shared__ __attribute__((aligned(16))) uint8_t s_txt[PW][WIN + PHALO + 16];
    /* the wave index stated wave-uniform (v_readfirstlane): derived from threadIdx, the
     * compiler's uniformity analysis takes it as lane-varying, and with it the file index,
     * the window position and every loop over them (exec-masked loops, state in VGPRs) */
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wv = PARSE_UNI ? (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) : threadIdx.x >> 6;
    uint8_t *const st = s_txt[wv];
    /* FAST: every file; EXACT: the files FAST abandoned (flist[0 .. *fcount)) */
    const uint64_t nf = FAST ? n_files : (uint64_t)*fcount;
    for (uint64_t k = (uint64_t)blockIdx.x * PW + wv; k < nf; k += (uint64_t)gridDim.x * PW) {
        const uint64_t f = FAST ? k : (uint64_t)flist[k];
        const uint64_t b0 = off[f], b1 = off[f + 1];
        uint16_t *const out = traces + f * stride;
        const uint64_t wbeg = b0 & ~15ull;
        const uint64_t last = b1 > wbeg ? ((b1 - 1) & ~15ull) : wbeg;     /* last in-file block */
        /* window loads: always issued (address clamped into the file) so they land straight
         * in their registers; bytes outside the file are masked by position */
        auto load = [&](uint64_t wa, uint4 (&v)[K], uint4 &h) {
#pragma unroll
            for (uint32_t k = 0; k < K; ++k) {
                const uint64_t q = wa + BPL * lane + 16u * k;
                v[k] = ldg16(text + (q < last ? q : last));
            }
            const uint64_t hq = wa + WIN + 16u * (lane & 1u);
            h = ldg16(text + (hq < last ? hq : last));
        };
        /* positions below are 32-bit, relative to wbeg (files are < 4 GiB) */
        const uint32_t s0 = (uint32_t)(b0 - wbeg), e0 = (uint32_t)(b1 - wbeg);   /* file [s0, e0) */
        uint32_t ls_rel = s0;         /* start of the line open at the window start          */
        uint32_t idx0 = 0;            /* chunks before the window                           */
        uint32_t err = 0xFFFFFFFFu;   /* first failing chunk: index * 8 + error class        */
        bool bad = false;             /* FAST: the file needs the EXACT pass                  */
        uint4 va[K], vb[K], ha, hb;
        uint64_t wa = wbeg;
        bool more = wbeg < b1;
        uint32_t psum = 0;            /* PARSE_PROBE 2: keeps the decode live */
        if (more) load(wa, va, ha);
        auto window = [&](uint64_t wa, const uint4 (&v)[K], const uint4 &h) {
            /* (1) stage [wa, wa + WIN + PHALO) */
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#pragma unroll
            for (uint32_t k = 0; k < K; ++k) reinterpret_cast<uint4 *>(st)[K * lane + k] = v[k];
            if (lane < 2) reinterpret_cast<uint4 *>(st + WIN)[lane] = h;
            /* (2) newlines among this lane's in-file bytes */
            const uint32_t wr0 = (uint32_t)(wa - wbeg);
            const uint32_t base = wr0 + BPL * lane;
            const uint32_t lo = base < s0 ? s0 - base : 0u;                      /* < 16 */
            const uint32_t hi = base + BPL <= e0 ? BPL : (base < e0 ? e0 - base : 0u);
            const uint32_t fm = hi > lo ? (lowmask(hi) & ~lowmask(lo)) : 0u;
            uint32_t nl = 0;
#if PARSE_TRANSPOSE
            if (4 * K == 8) {
                /* word k's newline flags (bit 8i+7 of byte i) into bit 8i+k of one word, then
                 * that 4 x 8 bit matrix transposed to byte order (bit 4k+i) by four delta swaps
                 * (the index bits rotated by two): fewer VALU than packing word by word */
#pragma unroll
                for (uint32_t k = 0; k < 8; ++k) {
                    const uint4 &q = v[k >> 2];
                    const uint32_t wd = (k & 3) == 0 ? q.x : (k & 3) == 1 ? q.y : (k & 3) == 2 ? q.z : q.w;
                    const uint32_t t = wd ^ 0x0A0A0A0Au;
                    const uint32_t z = ~(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t | 0x7F7F7F7Fu);
                    nl |= z >> (7 - k);
                }
                uint32_t tt;
                tt = (nl ^ (nl >> 1)) & 0x22222222u;  nl ^= tt ^ (tt << 1);
                tt = (nl ^ (nl >> 7)) & 0x00AA00AAu;  nl ^= tt ^ (tt << 7);
                tt = (nl ^ (nl >> 2)) & 0x0C0C0C0Cu;  nl ^= tt ^ (tt << 2);
                tt = (nl ^ (nl >> 14)) & 0x0000CCCCu; nl ^= tt ^ (tt << 14);
            } else
#endif
#pragma unroll
            for (uint32_t k = 0; k < 4 * K; ++k) {       /* bytes == '\n', 4 at a time */
                const uint4 &q = v[k >> 2];
                const uint32_t wd = (k & 3) == 0 ? q.x : (k & 3) == 1 ? q.y : (k & 3) == 2 ? q.z : q.w;
                const uint32_t t = wd ^ 0x0A0A0A0Au;
                const uint32_t z = ~(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t | 0x7F7F7F7Fu);
                nl |= (((z >> 7) & 1u) | ((z >> 14) & 2u) | ((z >> 21) & 4u) | ((z >> 28) & 8u)) << (4 * k);
            }
            nl &= fm;
            /* (3) line start at this lane's first byte: max over lower lanes of (last nl + 1) */
            const uint32_t my = nl ? base + (31u - __builtin_clz(nl)) + 1u : 0u;
            const uint32_t incl = wave_incl_max(my);
            const uint32_t lsr = umax(DPP(incl, 0x138, 0xF, 0xF, true), ls_rel);  /* wave_shr:1 */
            /* (4) chunk starts: line starts, and every 19 bytes into a longer line */
            const uint32_t din = lo > 0 ? 0u : base - lsr;       /* distance from line start */
            const uint32_t fnl = nl ? __builtin_ctz(nl) : BPL - 1u;
            uint32_t cs = ((nl << 1) | (lo > 0 ? (1u << lo) : (din == 0 ? 1u : 0u))) & fm;
            /* a byte at distance >= 19 from its line start: either in the line open at the
             * lane start (din), or after a run of 19 non-newline bytes inside the lane */
            const uint32_t r = ~nl & fm;
            const uint32_t t1 = r & (r >> 1), t2 = t1 & (t1 >> 2), t4 = t2 & (t2 >> 4), t8 = t4 & (t4 >> 8);
            const bool run19 = BPL > DP_CHUNK && (t8 & (t1 >> 16) & (r >> 18)) != 0u;
            /* (lanes past the file's end have no bytes: fm == 0 keeps them out) */
            const bool longl = fm != 0u && ((lo == 0 && din + (fnl < BPL - 1u ? fnl : BPL - 1u) >= DP_CHUNK) || run19);
            if (FAST) {
                bad = __ballot(longl) != 0;              /* a long line: the EXACT pass */
                if (bad) return;
            } else if (longl) {
                uint32_t d = din % DP_CHUNK;
                cs = 0;
                for (uint32_t j = 0; j < BPL; ++j) {
                    const uint32_t in = (fm >> j) & 1u;
                    cs |= (uint32_t)(in && d == 0) << j;
                    d = ((nl >> j) & 1u) ? 0u : (d == DP_CHUNK - 1 ? 0u : d + in);
                }
            }
            /* (5) instruction indices: a wave prefix sum of the chunk starts per lane (window
             * order = instruction order) */
            const uint32_t nc = __builtin_popcount(cs);
            const uint32_t isum = wave_incl_sum(nc);
            const uint32_t T = __builtin_amdgcn_readlane(isum, 63);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            /* (6) each lane parses the chunks that start in its bytes, one per round, from
             * LDS, 2-byte stores at their instruction index */
            const uint32_t tmax = cap - idx0 < T ? cap - idx0 : T;
            const uint32_t rem = e0 - wr0;                       /* file bytes from wa on */
            /* the fast path only, in a tight loop; the chunks it declines (any other shape,
             * an address whose home is >= np) are marked in `slow` and, in the EXACT pass,
             * scanned exactly after the loop */
            uint32_t mcs = cs, t = isum - nc, slow = 0;
            if (FAST && PARSE_PROBE == 1) mcs = 0;
            while (__ballot((mcs != 0u) & (t < tmax))) {
                if ((mcs != 0u) & (t < tmax)) {
                    const uint32_t b = (uint32_t)__builtin_ctz(mcs), o = BPL * lane + b;
                    const uint32_t lim = rem - o < DP_CHUNK ? rem - o : DP_CHUNK;
                    uint32_t d0, d1, d2, d3;
                    if (FAST && PARSE_PROBE == 3) {
                        d0 = v[0].x ^ o; d1 = v[0].y ^ t; d2 = v[0].z; d3 = v[0].w;
                    } else {
                        const uint32_t *wd = reinterpret_cast<const uint32_t *>(st + (o & ~3u));
                        d0 = wd[0]; d1 = wd[1]; d2 = wd[2]; d3 = wd[3];
                    }
                    const uint32_t c0 = __builtin_amdgcn_alignbyte(d1, d0, o & 3u);
                    const uint32_t c1 = __builtin_amdgcn_alignbyte(d2, d1, o & 3u);
                    const uint32_t c2 = __builtin_amdgcn_alignbyte(d3, d2, o & 3u);
                    uint32_t pk = 0;
                    const bool ok = PARSE_FAST(c0, c1, c2, lim, &pk) & (((pk >> 12) & 7u) < (uint32_t)np);
                    if (FAST && PARSE_PROBE == 2) psum += ok ? pk : 1u;
                    else if (ok) out[idx0 + t] = (uint16_t)pk;
                    slow |= ok ? 0u : 1u << b;
                }
                mcs &= mcs - 1u;
                ++t;
            }
            if (FAST) {
                if (PARSE_PROBE < 2) bad = __ballot(slow != 0u) != 0;   /* declined: EXACT pass */
            } else if (__ballot(slow != 0u)) {
                for (uint32_t m = slow; m; m &= m - 1u) {
                    const uint32_t b = (uint32_t)__builtin_ctz(m), o = BPL * lane + b;
                    const uint32_t ti = isum - nc + (uint32_t)__builtin_popcount(cs & lowmask(b));
                    const uint32_t lim = rem - o < DP_CHUNK ? rem - o : DP_CHUNK;
                    uint32_t pk = 0, len = 0;
                    while (len < lim) { if (st[o + len++] == '\n') break; }
                    int rc = dp_parse_chunk_at([&](uint32_t i) -> uint32_t { return i < len ? (uint32_t)st[o + i] : 0u; }, &pk);
                    if (rc == 0 && ((pk >> 12) & 7u) >= (uint32_t)np) rc = DSM_E_RANGE;   /* home < np */
                    if (rc == 0) out[idx0 + ti] = (uint16_t)pk;
                    else {
                        const uint32_t e = (idx0 + ti) * 8u + (rc == DSM_E_FORMAT ? 1u : 2u);
                        err = e < err ? e : err;
                    }
                }
                if (__ballot(err != 0xFFFFFFFFu)) err = wave_min(err);
            }
            idx0 += T;
            ls_rel = umax(ls_rel, __builtin_amdgcn_readlane(incl, 63));
        };
        /* the next window's loads are unconditional (clamped): a conditional load makes the
         * waitcnt at the join assume it was not issued, i.e. wait for it right away */
        while (more) {
            const uint64_t wn = wa + WIN;
            load(wn, vb, hb);
            window(wa, va, ha);
            more = wn < b1 && idx0 < cap && err == 0xFFFFFFFFu && !bad;
            if (!more) break;
            wa = wn;
            const uint64_t wn2 = wa + WIN;
            load(wn2, va, ha);
            window(wa, vb, hb);
            more = wn2 < b1 && idx0 < cap && err == 0xFFFFFFFFu && !bad;
            wa = wn2;
        }
        if (FAST && PARSE_PROBE == 2 && psum == 0x9E3779B9u) out[lane] = 0;
        if (lane == 0) {
            if (FAST && bad) {
                flist[atomicAdd(fcount, 1u)] = (uint32_t)f;     /* to the EXACT pass */
            } else {
                uint32_t n = idx0 < cap ? idx0 : cap;
                int32_t sc = DSM_OK;
                if (err != 0xFFFFFFFFu && (err >> 3) < n) {
                    n = err >> 3;
                    sc = (err & 7u) == 1u ? DSM_E_FORMAT : DSM_E_RANGE;
                }
                counts[f] = n;
                if (status) status[f] = sc;
            }
        }
    }
}

/* ---- synthetic core files ("RD 0x%02x\n" / "WR 0x%02x %u\n", the shipped core_n.txt format) -- */
DEVI uint32_t text_line_len(uint32_t ins) {
    if (!(ins >> 15)) return 8u;
    const uint32_t v = ins & 0xFFu;
    return 10u + (v >= 10u) + (v >= 100u);
}
template <int NP>
__global__ void __launch_bounds__(256) textlen_kernel(uint64_t seed, int dist, uint64_t first,
                                                    uint64_t n_files, uint32_t n_instr,
                                                    uint64_t *lens) {
    const uint64_t gmul = seed * 0x9E3779B97F4A7C15ULL;
    for (uint64_t f = (uint64_t)blockIdx.x * 256 + threadIdx.x; f < n_files;
         f += (uint64_t)gridDim.x * 256) {
        uint64_t s = 0;
        for (uint32_t i = 0; i < n_instr; ++i)
            s += text_line_len(dsmg::gen_instr<NP>(gmul, dist, first + f / NP, (uint32_t)(f % NP), i));
        lens[f + 1] = s;
    }
}
/* exclusive scan of lens[1..n] into offsets (in place, offsets[0] = 0), one workgroup */
__global__ void __launch_bounds__(1024) scan_kernel(uint64_t *a, uint64_t n) {
    __shared__ uint64_t s[1024];
    const uint64_t per = (n + 1023) / 1024, lo = threadIdx.x * per;
    const uint64_t hi = lo + per < n ? lo + per : n;
    uint64_t t = 0;
    for (uint64_t i = lo; i < hi; ++i) t += a[i + 1];
    s[threadIdx.x] = t;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t acc = 0;
        for (int i = 0; i < 1024; ++i) { const uint64_t x = s[i]; s[i] = acc; acc += x; }
    }
    __syncthreads();
    uint64_t acc = s[threadIdx.x];
    for (uint64_t i = lo; i < hi; ++i) { const uint64_t x = a[i + 1]; a[i + 1] = acc + x; acc += x; }
    if (threadIdx.x == 0) a[0] = 0;
}
/* one wave per file, 64 lines per step; line bytes written one at a time (setup, not timed) */
template <int NP>
__global__ void __launch_bounds__(256) textgen_kernel(uint64_t seed, int dist, uint64_t first,
                                                    uint64_t n_files, uint32_t n_instr,
                                                    const uint64_t *off, uint8_t *text) {
    const uint64_t gmul = seed * 0x9E3779B97F4A7C15ULL;
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    for (uint64_t f = (uint64_t)blockIdx.x * 4 + wv; f < n_files; f += (uint64_t)gridDim.x * 4) {
        uint64_t pos = off[f];
        for (uint32_t i0 = 0; i0 < n_instr; i0 += 64) {
            const uint32_t i = i0 + lane;
            const bool ok = i < n_instr;
            const uint32_t ins = ok ? dsmg::gen_instr<NP>(gmul, dist, first + f / NP, (uint32_t)(f % NP), i) : 0u;
            const uint32_t len = ok ? text_line_len(ins) : 0u;
            const uint32_t inc = wave_incl_sum(len);
            uint8_t *q = text + pos + (inc - len);
            if (ok) {
                const uint32_t a = (ins >> 8) & 0x7Fu, v = ins & 0xFFu;
                const bool wr = ins >> 15;
                q[0] = wr ? 'W' : 'R'; q[1] = wr ? 'R' : 'D'; q[2] = ' '; q[3] = '0'; q[4] = 'x';
                q[5] = (uint8_t)"0123456789abcdef"[a >> 4]; q[6] = (uint8_t)"0123456789abcdef"[a & 15u];
                if (!wr) q[7] = '\n';
                else {
                    q[7] = ' ';
                    uint32_t k = 8;
                    if (v >= 100u) q[k++] = (uint8_t)('0' + v / 100u);
                    if (v >= 10u) q[k++] = (uint8_t)('0' + (v / 10u) % 10u);
                    q[k++] = (uint8_t)('0' + v % 10u);
                    q[k] = '\n';
                }
            }
            pos += __shfl(inc, 63, 64);
        }
    }
}

}  // namespace

/* ====================================================================================== */

void dsm_text_release(dsm_ctx *c) {
    void *ptrs[] = {c->d_dump_tpl, c->d_text_tmp, c->d_len_tmp, c->d_parse_buf, c->d_parse_off,
                    c->d_parse_list};
    for (void *p : ptrs) if (p) (void)hipFree(p);
}

/* np templates: the reference text of an all-zero record, zero-padded to DSM_DUMP_SLOT */
static int ensure_templates(dsm_ctx *c) {
    if (c->d_dump_tpl) return DSM_OK;
    const int np = c->cfg.np;
    char *h = (char *)calloc((size_t)np, SLOT);
    if (!h) return DSM_E_NOMEM;
    dsm_node_state z;
    memset(&z, 0, sizeof z);
    for (int n = 0; n < np; ++n) {
        const int len = dsm_format_dump(n, &z, h + (size_t)n * SLOT, SLOT);
        if (len != DSM_DUMP_BASE) { free(h); return DSM_E_STATE; }
        h[(size_t)n * SLOT + len] = 0;
    }
    uint4 *d = nullptr;
    if (hipMalloc((void **)&d, (size_t)np * SLOT) != hipSuccess) { free(h); return DSM_E_NOMEM; }
    const bool ok = hipMemcpy(d, h, (size_t)np * SLOT, hipMemcpyHostToDevice) == hipSuccess;
    free(h);
    if (!ok) { (void)hipFree(d); return DSM_E_DEVICE; }
    c->d_dump_tpl = d;
    return DSM_OK;
}

/* Workgroup tile of fmt_kernel: DSM_FMT=FR (4, 8, 16: records per iteration, templates read
 * from L2) or 100 + FR (108, 116, 132: templates resident in LDS, next tile's records
 * prefetched) for A/B runs.  Measured on 8M records (tools/ab_fmt.py): 16 5.47 ms, 116 3.40,
 * 132 3.35 (5.1 TB/s) -- the default. */
static int fmt_choice(const dsm_ctx *c) {      /* c->fmt_tile: DSM_FMT, read at dsm_open */
    const int v = c->fmt_tile;
    return (v == 4 || v == 8 || v == 16 || v == 108 || v == 116) ? v : 132;   /* 1xx: LDS templates */
}

static int launch_fmt(dsm_ctx *c, const uint8_t *recs, uint64_t stride_bytes, uint64_t n,
                      char *d_text, uint32_t *d_len, hipStream_t st) {
    if (n == 0) return DSM_OK;
    int rc = ensure_templates(c);
    if (rc) return rc;
    const int v = fmt_choice(c), fr = v % 100;
    const bool tl = v >= 100;
    const void *fn = tl ? (fr == 8 ? (const void *)fmt_kernel<8, 128, true>
                           : fr == 32 ? (const void *)fmt_kernel<32, 512, true> : (const void *)fmt_kernel<16, 256, true>)
                        : fr == 4 ? (const void *)fmt_kernel<4, 64, false>
                        : fr == 8 ? (const void *)fmt_kernel<8, 128, false> : (const void *)fmt_kernel<16, 256, false>;
    const int nt = fr == 4 ? 64 : fr == 8 ? 128 : fr == 32 ? 512 : 256;
    int per_cu = 0;
    HIPCK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, nt, 0));
    if (per_cu < 1) per_cu = 1;
    uint64_t blocks = (n + fr - 1) / fr;
    const uint64_t cap = (uint64_t)c->cus * per_cu;             /* one resident round */
    if (blocks > cap) blocks = cap;
    const uint4 *tpl = (const uint4 *)c->d_dump_tpl;
    v4u32 *out = (v4u32 *)d_text;
    hipLaunchKernelGGL(reinterpret_cast<void (*)(const uint8_t *, uint64_t, uint64_t, int, const uint4 *, v4u32 *, uint32_t *)>(const_cast<void *>(fn)),
                       dim3((unsigned)blocks), dim3(nt), 0, st, recs, stride_bytes, n, c->cfg.np, tpl, out, d_len);
    HIPCK(hipGetLastError());
    return DSM_OK;
}

extern "C" int dsm_format_dumps_device(dsm_ctx *c, const dsm_node_state *d_states,
                                       uint32_t state_stride, uint64_t n_states, char *d_text,
                                       uint32_t *d_len, void *stream) {
    if (!c || state_stride == 0 || (n_states && (!d_states || !d_text || !d_len))) return DSM_E_INVAL;
    if (((uintptr_t)d_text & 15u) || ((uintptr_t)d_states & 15u)) return DSM_E_INVAL;
    HIPCK(hipSetDevice(c->device));
    return launch_fmt(c, (const uint8_t *)d_states, (uint64_t)state_stride * sizeof(dsm_node_state),
                      n_states, d_text, d_len, (hipStream_t)stream);
}

extern "C" int dsm_format_run_dumps_device(dsm_ctx *c, int view, uint64_t first_sys,
                                           uint64_t n_sys, char *d_text, uint32_t *d_len,
                                           void *stream) {
    if (!c || (view != DSM_VIEW_DUMP && view != DSM_VIEW_FINAL)) return DSM_E_INVAL;
    if (!c->d_recs) return DSM_E_STATE;
    if (first_sys > c->recs_n || n_sys > c->recs_n - first_sys) return DSM_E_INVAL;
    if (n_sys && (!d_text || !d_len || ((uintptr_t)d_text & 15u))) return DSM_E_INVAL;
    HIPCK(hipSetDevice(c->device));
    const uint8_t *recs = (const uint8_t *)c->d_recs + first_sys * (uint64_t)c->cfg.np * 128 + view * 64;
    return launch_fmt(c, recs, 128, n_sys * (uint64_t)c->cfg.np, d_text, d_len, (hipStream_t)stream);
}

extern "C" int dsm_write_run_dumps(dsm_ctx *c, uint64_t sys, uint32_t node_mask, const char *dir) {
    if (!c) return DSM_E_INVAL;
    if (!(c->cfg.flags & DSM_F_SNAPSHOTS) || !c->d_recs) return DSM_E_STATE;
    if (sys >= c->recs_n) return DSM_E_INVAL;
    const int np = c->cfg.np;
    HIPCK(hipSetDevice(c->device));
    if (!c->d_text_tmp) HIPCK(hipMalloc((void **)&c->d_text_tmp, (size_t)DSM_MAX_NP * SLOT));
    if (!c->d_len_tmp) HIPCK(hipMalloc((void **)&c->d_len_tmp, DSM_MAX_NP * sizeof(uint32_t)));
    int rc = dsm_format_run_dumps_device(c, DSM_VIEW_DUMP, sys, 1, c->d_text_tmp, c->d_len_tmp, c->stream);
    if (rc) return rc;
    char *h = (char *)malloc((size_t)np * SLOT);
    uint32_t lens[DSM_MAX_NP];
    if (!h) return DSM_E_NOMEM;
    if (hipMemcpyAsync(h, c->d_text_tmp, (size_t)np * SLOT, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
        hipMemcpyAsync(lens, c->d_len_tmp, np * sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess) {
        free(h);
        return DSM_E_DEVICE;
    }
    rc = DSM_OK;
    for (int n = 0; n < np && rc == DSM_OK; ++n) {
        if (!((node_mask >> n) & 1u)) continue;
        char path[512];
        if (dir) snprintf(path, sizeof path, "%s/core_%d_output.txt", dir, n);
        else snprintf(path, sizeof path, "core_%d_output.txt", n);            /* :831 */
        FILE *f = fopen(path, "w");
        if (!f) { rc = DSM_E_IO; break; }
        const size_t w = fwrite(h + (size_t)n * SLOT, 1, lens[n], f);
        if (fclose(f) != 0 || w != lens[n]) rc = DSM_E_IO;
    }
    free(h);
    return rc;
}

/* ---- trace parser / text generator ABI ---------------------------------------------- */
extern "C" int dsm_parse_traces_device(dsm_ctx *c, const char *d_text, const uint64_t *d_offsets,
                                       uint64_t n_files, uint32_t cap, uint16_t *d_traces,
                                       uint32_t *d_counts, int32_t *d_status, void *stream) {
    if (!c || cap > c->cfg.max_instr) return DSM_E_INVAL;
    if (n_files && (!d_text || !d_offsets || !d_traces || !d_counts)) return DSM_E_INVAL;
    if (n_files == 0) return DSM_OK;
    if (n_files > 0xFFFFFFFFull) return DSM_E_INVAL;
    HIPCK(hipSetDevice(c->device));
    hipStream_t st = (hipStream_t)stream;
    /* the EXACT pass's file list: [0] = count, then file ids */
    int rc = dsm_ensure(&c->d_parse_list, &c->parse_list_cap, (size_t)n_files + 1);
    if (rc) return rc;
    HIPCK(hipMemsetAsync(c->d_parse_list, 0, sizeof(uint32_t), st));
    /* DSM_PARSE_BPL=16|32 (read at dsm_open): bytes per lane per window (1 or 2 KB
     * windows), for A/B runs */
    const bool b32 = c->parse_bpl != 16;
    const void *fast = b32 ? (const void *)parse_kernel<32, true> : (const void *)parse_kernel<16, true>;
    /* one resident round of workgroups: a grid-stride loop over files with a second, partial
     * round of workgroups would leave most of the chip idle at the end */
    int per_cu = 0;
    HIPCK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fast, 64 * PW, 0));
    if (per_cu < 1) per_cu = 1;
    uint64_t blocks = (n_files + PW - 1) / PW;
    const uint64_t lim = (uint64_t)c->cus * per_cu;
    if (blocks > lim) blocks = lim;
    uint32_t *fl = c->d_parse_list + 1, *fc = c->d_parse_list;
    const uint8_t *tx = (const uint8_t *)d_text;
    const uint32_t mi = c->cfg.max_instr;
    const int np = c->cfg.np;
    /* the FAST pass over every file, then the EXACT pass over the files it listed (sized on
     * the device: its workgroups past the list's count exit at once) */
    if (b32) {
        hipLaunchKernelGGL((parse_kernel<32, true>), dim3((unsigned)blocks), dim3(64 * PW), 0, st,
                           tx, d_offsets, n_files, cap, mi, np, d_traces, d_counts, d_status, fl, fc);
        hipLaunchKernelGGL((parse_kernel<32, false>), dim3((unsigned)blocks), dim3(64 * PW), 0, st,
                           tx, d_offsets, n_files, cap, mi, np, d_traces, d_counts, d_status, fl, fc);
    } else {
        hipLaunchKernelGGL((parse_kernel<16, true>), dim3((unsigned)blocks), dim3(64 * PW), 0, st,
                           tx, d_offsets, n_files, cap, mi, np, d_traces, d_counts, d_status, fl, fc);
        hipLaunchKernelGGL((parse_kernel<16, false>), dim3((unsigned)blocks), dim3(64 * PW), 0, st,
                           tx, d_offsets, n_files, cap, mi, np, d_traces, d_counts, d_status, fl, fc);
    }
    HIPCK(hipGetLastError());
    return DSM_OK;
}

extern "C" int dsm_parse_traces(dsm_ctx *c, const char *text, const uint64_t *offsets,
                                uint64_t n_files, uint32_t cap, uint16_t *traces,
                                uint32_t *counts, int32_t *status) {
    if (!c || (n_files && (!text || !offsets || !traces || !counts))) return DSM_E_INVAL;
    if (n_files == 0) return DSM_OK;
    const uint64_t bytes = offsets[n_files] - offsets[0];
    for (uint64_t f = 0; f < n_files; ++f)
        if (offsets[f + 1] < offsets[f]) return DSM_E_INVAL;
    HIPCK(hipSetDevice(c->device));
    const uint32_t stride = c->cfg.max_instr;
    char *d_text = nullptr;
    uint64_t *d_off = nullptr;
    uint16_t *d_tr = nullptr;
    uint32_t *d_cn = nullptr;
    int32_t *d_st = nullptr;
    uint64_t *h_off = (uint64_t *)malloc((n_files + 1) * sizeof(uint64_t));
    int rc = h_off ? DSM_OK : DSM_E_NOMEM;
    if (rc == DSM_OK) {
        for (uint64_t f = 0; f <= n_files; ++f) h_off[f] = offsets[f] - offsets[0];
        if (hipMalloc((void **)&d_text, bytes + 64) != hipSuccess ||
            hipMalloc((void **)&d_off, (n_files + 1) * sizeof(uint64_t)) != hipSuccess ||
            hipMalloc((void **)&d_tr, n_files * stride * sizeof(uint16_t)) != hipSuccess ||
            hipMalloc((void **)&d_cn, n_files * sizeof(uint32_t)) != hipSuccess ||
            hipMalloc((void **)&d_st, n_files * sizeof(int32_t)) != hipSuccess)
            rc = DSM_E_NOMEM;
    }
    if (rc == DSM_OK &&
        (hipMemcpyAsync(d_text, text + offsets[0], bytes, hipMemcpyHostToDevice, c->stream) != hipSuccess ||
         hipMemcpyAsync(d_off, h_off, (n_files + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, c->stream) != hipSuccess))
        rc = DSM_E_DEVICE;
    if (rc == DSM_OK) rc = dsm_parse_traces_device(c, d_text, d_off, n_files, cap, d_tr, d_cn, d_st, c->stream);
    if (rc == DSM_OK &&
        (hipMemcpyAsync(traces, d_tr, n_files * stride * sizeof(uint16_t), hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
         hipMemcpyAsync(counts, d_cn, n_files * sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
         (status && hipMemcpyAsync(status, d_st, n_files * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream) != hipSuccess) ||
         hipStreamSynchronize(c->stream) != hipSuccess))
        rc = DSM_E_DEVICE;
    (void)hipStreamSynchronize(c->stream);
    void *ptrs[] = {d_text, d_off, d_tr, d_cn, d_st};
    for (void *p : ptrs) if (p) (void)hipFree(p);
    free(h_off);
    return rc;
}

extern "C" int dsm_generate_text_device(dsm_ctx *c, const dsm_gen *g, uint64_t first_sys,
                                        uint64_t n_sys, char *d_text, uint64_t *d_offsets,
                                        void *stream) {
    if (!c || !g || !d_offsets || g->dist < 0 || g->dist > 2 || g->n_instr > DSM_MAX_INSTR) return DSM_E_INVAL;
    HIPCK(hipSetDevice(c->device));
    const uint64_t n = n_sys * (uint64_t)c->cfg.np;
    hipStream_t st = (hipStream_t)stream;
    uint64_t blocks = (n + 255) / 256;
    if (blocks > (uint64_t)c->cus * 8) blocks = (uint64_t)c->cus * 8;
    if (blocks == 0) blocks = 1;
    if (c->cfg.np == 4)
        hipLaunchKernelGGL(textlen_kernel<4>, dim3((unsigned)blocks), dim3(256), 0, st, g->seed, g->dist, first_sys, n, g->n_instr, d_offsets);
    else
        hipLaunchKernelGGL(textlen_kernel<8>, dim3((unsigned)blocks), dim3(256), 0, st, g->seed, g->dist, first_sys, n, g->n_instr, d_offsets);
    hipLaunchKernelGGL(scan_kernel, dim3(1), dim3(1024), 0, st, d_offsets, n);
    HIPCK(hipGetLastError());
    if (!d_text) return DSM_OK;
    uint64_t wblocks = (n + 3) / 4;
    if (wblocks > (uint64_t)c->cus * 16) wblocks = (uint64_t)c->cus * 16;
    if (wblocks == 0) wblocks = 1;
    if (c->cfg.np == 4)
        hipLaunchKernelGGL(textgen_kernel<4>, dim3((unsigned)wblocks), dim3(256), 0, st, g->seed, g->dist, first_sys, n, g->n_instr, (const uint64_t *)d_offsets, (uint8_t *)d_text);
    else
        hipLaunchKernelGGL(textgen_kernel<8>, dim3((unsigned)wblocks), dim3(256), 0, st, g->seed, g->dist, first_sys, n, g->n_instr, (const uint64_t *)d_offsets, (uint8_t *)d_text);
    HIPCK(hipGetLastError());
    return DSM_OK;
}
