/*
 * dsm_gen.h -- the counter-based synthetic trace generator (device side), shared by the
 * transition kernel (fused mode), gen_kernel and the text generator.  Definition in
 * DESIGN.md; pinned against oracle/dsm_common.h by the tests.
 */
#ifndef DSM_GEN_H
#define DSM_GEN_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dsm.h"

namespace dsmg {

__device__ __forceinline__ uint64_t splitmix(uint64_t z) {
    z += 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
/* One splitmix64 output feeds 4 consecutive instructions, 16 bits each. */
template <int NP>
__device__ __forceinline__ uint32_t instr_from_bits(uint32_t h, int dist) {
    const uint32_t wr = h & 1u;
    const uint32_t val = (h >> 1) & (0u - wr) & 0xFFu;          /* RD: value 0 */
    const uint32_t sel = h >> 9;
    uint32_t addr;
    if (dist == DSM_DIST_HOT) addr = (sel & 3u) * 0x11u;
    else if (dist == DSM_DIST_EVICT) addr = (sel & (uint32_t)(NP * 4 - 1)) * 4u;
    else addr = sel & (uint32_t)(NP * 16 - 1);
    return (wr << 15) | (addr << 8) | val;
}
template <int NP>
__device__ __forceinline__ uint32_t gen_instr(uint64_t gmul, int dist, uint64_t sys, uint32_t node, uint32_t idx) {
    const uint64_t key = (sys << 16) | ((uint64_t)node << 12) | (uint64_t)((idx & 0xFFFu) >> 2);
    const uint64_t r = splitmix(gmul + key);
    return instr_from_bits<NP>((uint32_t)(r >> (16 * (idx & 3u))) & 0xFFFFu, dist);
}

}  // namespace dsmg

#endif
