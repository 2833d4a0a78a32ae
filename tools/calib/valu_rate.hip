// tools/calib/valu_rate.hip -- throughput of single VALU instructions on gfx950 (wave64, SIMD-32),
// to price the transition kernels' instruction mix: each lane runs 8 independent chains of one
// instruction (inline asm, so nothing is folded), at 8 waves per SIMD; prints cycles per
// wave-instruction per SIMD (2 = full rate, 4 = half rate).  Vector registers only; the one
// store per lane keeps the chains live.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define ITERS 4096

#define BODY(ASM)                                                                      \
    __global__ void __launch_bounds__(512) k_##ASM(unsigned *out, unsigned seed) {     \
        unsigned a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;        \
        unsigned a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;                    \
        const unsigned b = seed * 7u + 3u, c = seed * 13u + 5u;                          \
        const unsigned sb = __builtin_amdgcn_readfirstlane(b);                           \
        const unsigned long long msk = __builtin_amdgcn_ballot_w64(a0 & 1u);             \
        unsigned long long msk2 = 0;                                                     \
        for (int i = 0; i < ITERS; ++i) {                                               \
            ASM(a0); ASM(a1); ASM(a2); ASM(a3); ASM(a4); ASM(a5); ASM(a6); ASM(a7);     \
        }                                                                              \
        out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ (unsigned)msk2; \
    }

#define ADD(x) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(b))
#define AND(x) asm volatile("v_and_b32 %0, %0, %1" : "+v"(x) : "v"(b))
#define PERM(x) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c))
#define BFE(x) asm volatile("v_bfe_u32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c))
#define LSHLOR(x) asm volatile("v_lshl_or_b32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c))
#define ANDOR(x) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c))
#define ALIGNB(x) asm volatile("v_alignbit_b32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c))
#define BITOP3(x) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x) : "v"(b), "v"(c))
#define OR3(x) asm volatile("v_or3_b32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c))
#define ADD3(x) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c))
#define FFBL(x) asm volatile("v_ffbl_b32 %0, %0" : "+v"(x))
#define BCNT(x) asm volatile("v_bcnt_u32_b32 %0, %0, %1" : "+v"(x) : "v"(b))
#define CNDM(x) asm volatile("v_cmp_gt_u32 vcc, %0, %1\n\tv_cndmask_b32 %0, %0, %1, vcc" : "+v"(x) : "v"(b) : "vcc")
#define MULLO(x) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x) : "v"(b))
#define CNDM64(x) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(x) : "v"(b), "s"(msk))
#define CMP64(x) asm volatile("v_cmp_gt_u32_e64 %0, %1, %2" : "=s"(msk2) : "v"(x), "v"(b)); x += 0
#define BFEI(x) asm volatile("v_bfe_i32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c))
#define LSHLADD(x) asm volatile("v_lshl_add_u32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c))
#define LSHLS(x) asm volatile("v_lshlrev_b32_e64 %0, %1, %0" : "+v"(x) : "s"(sb))
#define MINU(x) asm volatile("v_min_u32 %0, %0, %1" : "+v"(x) : "v"(b))
#define LSHR(x) asm volatile("v_lshrrev_b32 %0, %1, %0" : "+v"(x) : "v"(b))
#define XOR3(x) asm volatile("v_xor3_b32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c))
#define BITOP3S(x) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xe8" : "+v"(x) : "s"(sb), "v"(c))
#define SHR64(x) asm volatile("v_lshrrev_b64 %0, %1, %0" : "+v"(x##w) : "v"(b))
#define ANDLIT(x) asm volatile("v_and_b32_e32 %0, 0x12345, %0" : "+v"(x))
#define ANDS(x) asm volatile("v_and_b32_e32 %0, %1, %0" : "+v"(x) : "s"(sb))
#define ADDS(x) asm volatile("v_add_u32_e32 %0, %1, %0" : "+v"(x) : "s"(sb))
#define CNDVCC(x) asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(x) : "v"(b))
#define CMPVCC(x) asm volatile("v_cmp_gt_u32_e32 vcc, %0, %1" : : "v"(x), "v"(b) : "vcc"); x += 0
#define BITOP3I(x) asm volatile("v_bitop3_b32 %0, %0, 7, %1 bitop3:0xe8" : "+v"(x) : "v"(c))
#define PERMS(x) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "s"(sb))
#define MOVV(x) asm volatile("v_mov_b32 %0, %1" : "=v"(x) : "v"(b)); x += 0
#define NOTB(x) asm volatile("v_not_b32 %0, %0" : "+v"(x))
#define SDWA(x) asm volatile("v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD" : "+v"(x) : "v"(b))

BODY(ADD) BODY(AND) BODY(PERM) BODY(BFE) BODY(LSHLOR) BODY(ANDOR) BODY(ALIGNB) BODY(BITOP3)
BODY(OR3) BODY(ADD3) BODY(FFBL) BODY(BCNT) BODY(CNDM) BODY(MULLO) BODY(SDWA)
BODY(CNDM64) BODY(CMP64) BODY(BFEI) BODY(LSHLADD) BODY(LSHLS) BODY(MINU) BODY(LSHR) BODY(BITOP3S)
BODY(ANDLIT) BODY(ANDS) BODY(ADDS) BODY(CNDVCC) BODY(CMPVCC) BODY(BITOP3I) BODY(PERMS) BODY(NOTB)

typedef void (*kfn)(unsigned *, unsigned);
struct K { const char *name; kfn f; int per; };

int main() {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, 0) != hipSuccess) return 1;
    const int cus = p.multiProcessorCount;
    const int blocks = cus * 4;                 /* 4 x 512 threads = 32 waves per CU = 8 per SIMD */
    unsigned *out;
    if (hipMalloc(&out, (size_t)blocks * 512 * 4) != hipSuccess) return 1;
    K ks[] = {{"v_add_u32", k_ADD, 1}, {"v_and_b32", k_AND, 1}, {"v_perm_b32", k_PERM, 1},
              {"v_bfe_u32", k_BFE, 1}, {"v_lshl_or_b32", k_LSHLOR, 1}, {"v_and_or_b32", k_ANDOR, 1},
              {"v_alignbit_b32", k_ALIGNB, 1}, {"v_bitop3_b32", k_BITOP3, 1}, {"v_or3_b32", k_OR3, 1},
              {"v_add3_u32", k_ADD3, 1}, {"v_ffbl_b32", k_FFBL, 1}, {"v_bcnt_u32_b32", k_BCNT, 1},
              {"v_cmp+v_cndmask", k_CNDM, 2}, {"v_mul_lo_u32", k_MULLO, 1}, {"v_add_u32_sdwa", k_SDWA, 1},
              {"v_cndmask_b32_e64 (sgpr mask)", k_CNDM64, 1}, {"v_cmp_gt_u32_e64 (to sgpr)", k_CMP64, 1},
              {"v_bfe_i32", k_BFEI, 1}, {"v_lshl_add_u32", k_LSHLADD, 1}, {"v_lshlrev_b32_e64 (sgpr)", k_LSHLS, 1},
              {"v_min_u32", k_MINU, 1}, {"v_lshrrev_b32", k_LSHR, 1},
              {"v_bitop3_b32 (sgpr)", k_BITOP3S, 1},
              {"v_and_b32_e32 (literal)", k_ANDLIT, 1}, {"v_and_b32_e32 (sgpr)", k_ANDS, 1},
              {"v_add_u32_e32 (sgpr)", k_ADDS, 1}, {"v_cndmask_b32_e32 (vcc)", k_CNDVCC, 1},
              {"v_cmp_gt_u32_e32 (to vcc)", k_CMPVCC, 1}, {"v_bitop3_b32 (inline const)", k_BITOP3I, 1},
              {"v_perm_b32 (sgpr selector)", k_PERMS, 1}, {"v_not_b32", k_NOTB, 1}};
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    int clk = 0;
    hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);   /* kHz */
    printf("{\"cus\": %d, \"clock_khz\": %d, \"waves_per_simd\": 8, \"results\": [\n", cus, clk);
    for (size_t i = 0; i < sizeof ks / sizeof ks[0]; ++i) {
        hipLaunchKernelGGL(ks[i].f, dim3(blocks), dim3(512), 0, 0, out, 1u);   /* warm */
        hipEventRecord(e0, 0);
        for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(ks[i].f, dim3(blocks), dim3(512), 0, 0, out, (unsigned)r);
        hipEventRecord(e1, 0);
        if (hipEventSynchronize(e1) != hipSuccess) return 1;
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        /* wave-instructions per SIMD: 8 waves x ITERS x 8 chains x per, 5 launches */
        const double winst = 8.0 * ITERS * 8 * ks[i].per * 5;
        const double cyc = ms * 1e-3 * clk * 1e3;
        printf("  {\"op\": \"%s\", \"ms\": %.3f, \"cycles_per_wave_instr\": %.2f}%s\n", ks[i].name, ms,
               cyc / winst, i + 1 < sizeof ks / sizeof ks[0] ? "," : "");
    }
    printf("]}\n");
    hipFree(out);
    return 0;
}
