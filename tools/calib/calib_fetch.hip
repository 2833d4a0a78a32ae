// tools/calib/calib_fetch.hip -- calibrates rocprofv3 FETCH_SIZE for the transition kernels'
// trace access pattern (not product): every lane reads its own node slot (8 KiB apart, as
// [sys][node][4096] u16 traces) as consecutive 16-byte chunks, one chunk per loop iteration
// with dependent ALU work in between, so a slot's chunks are requested thousands of cycles
// apart.  Prints the bytes requested; compare with FETCH_SIZE of the same run.
//   hipcc --offload-arch=gfx950 -O3 tools/calib/calib_fetch.hip -o ab/calib_fetch
//   rocprofv3 --pmc FETCH_SIZE -- ab/calib_fetch <lanes> <chunks per lane> <alu per chunk>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

__global__ void __launch_bounds__(256) calib(const uint4 *slots, uint32_t chunks, uint32_t alu,
                                              uint32_t *sink) {
    const uint64_t lane = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const uint4 *p = slots + lane * 512;          /* 8 KiB per lane = 512 chunks */
    uint32_t acc = (uint32_t)lane;
    for (uint32_t c = 0; c < chunks; ++c) {
        const uint4 v = p[c];
        acc ^= v.x + v.y + v.z + v.w;
        for (uint32_t k = 0; k < alu; ++k) acc = acc * 0x9E3779B1u + k;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

int main(int argc, char **argv) {
    const uint64_t lanes = argc > 1 ? strtoull(argv[1], 0, 10) : (1ull << 20);
    const uint32_t chunks = argc > 2 ? (uint32_t)atoi(argv[2]) : 16;
    const uint32_t alu = argc > 3 ? (uint32_t)atoi(argv[3]) : 64;
    uint4 *d = nullptr;
    uint32_t *sink = nullptr;
    if (hipMalloc((void **)&d, lanes * 8192) != hipSuccess || hipMalloc((void **)&sink, 4) != hipSuccess) return 1;
    if (hipMemset(d, 1, lanes * 8192) != hipSuccess) return 1;
    hipLaunchKernelGGL(calib, dim3((unsigned)(lanes / 256)), dim3(256), 0, 0, d, chunks, alu, sink);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    printf("{\"lanes\": %llu, \"chunks\": %u, \"alu\": %u, \"bytes_requested\": %llu}\n",
           (unsigned long long)lanes, chunks, alu, (unsigned long long)(lanes * chunks * 16ull));
    (void)hipFree(d);
    (void)hipFree(sink);
    return 0;
}
