/* tests/native/parse_fast_equiv.cpp -- host check that parse_fast_v3 (the chunk loop's decoder) and
 * parse_fast_swar accept exactly the chunks the byte-wise parse_fast accepts, with the same packed
 * instruction, on canonical
 * "RD 0xHH\n" / "WR 0xHH D\n" lines mutated at random (tests/test_parse_swar.py). */
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#define DEVI static inline
static inline uint32_t __builtin_amdgcn_ubfe(uint32_t w, uint32_t o, uint32_t n) { return (w >> o) & ((1u << n) - 1u); }
#include "pf.h"   /* parse_fast .. parse_fast_swar, cut from csrc/dsm_text.hip by the test */
static uint32_t W(const unsigned char *b, int i) { uint32_t x; memcpy(&x, b + i, 4); return x; }
int main() {
    std::mt19937_64 g(1);
    const char alpha[] = "RDW x0123456789abcdefABCDEFgG\n\r\t-+:9";
    long n = 0, acc = 0;
    auto check = [&](const unsigned char *b, uint32_t lim) {
        uint32_t p1 = 0, p2 = 0;
        uint32_t o1 = parse_fast(W(b,0), W(b,4), W(b,8), lim, &p1);
        uint32_t o2 = parse_fast_swar(W(b,0), W(b,4), W(b,8), lim, &p2);
        uint32_t p3 = 0;
        uint32_t o3 = parse_fast_v3(W(b,0), W(b,4), W(b,8), lim, &p3);
        ++n; acc += o1;
        if (o1 != o3 || (o1 && p1 != p3)) { printf("MISMATCH v3 o %u %u pk %x %x lim %u:", o1, o3, p1, p3, lim); for (int k = 0; k < 12; ++k) printf(" %02x", b[k]); printf("\n"); return false; }
        if (o1 != o2 || (o1 && p1 != p2)) { printf("MISMATCH o %u %u pk %x %x lim %u:", o1, o2, p1, p2, lim); for (int k = 0; k < 12; ++k) printf(" %02x", b[k]); printf("\n"); return false; }
        return true;
    };
    unsigned char b[16];
    for (long it = 0; it < 4000000; ++it) {
        // structured: start from a canonical line and mutate a few bytes
        uint32_t a = g() & 0xFF, v = g() % 1000; int wr = g() & 1;
        char s[32];
        int len = wr ? snprintf(s, sizeof s, "WR 0x%02x %u\n", a, v) : snprintf(s, sizeof s, "RD 0x%02X\n", a);
        memset(b, 0, 16); memcpy(b, s, len < 16 ? len : 16);
        for (int k = len; k < 16; ++k) b[k] = alpha[g() % (sizeof alpha - 1)];
        int nm = g() % 4;
        for (int k = 0; k < nm; ++k) { int pos = g() % 12; b[pos] = (g() & 3) ? alpha[g() % (sizeof alpha - 1)] : (unsigned char)g(); }
        uint32_t lim = (g() & 3) ? 19 : g() % 20;
        if (!check(b, lim)) return 1;
    }
    printf("ok %ld cases, %ld accepted\n", n, acc);
}
