// tools/calib/lds_unaligned.hip -- does a ds_read_b32 / ds_read_b64 at an address that is not a
// multiple of 4 return the unaligned bytes on gfx950 (the parser's chunk gathers could then
// drop their v_alignbyte_b32s), and what does it cost: the bytes read at offsets 0..7, and the
// time of 64K unaligned vs aligned reads per wave.  LDS and vector registers only.
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void k_check(unsigned *out) {
    __shared__ unsigned char b[256];
    for (int i = threadIdx.x; i < 256; i += 64) b[i] = (unsigned char)i;
    __syncthreads();
    const unsigned off = threadIdx.x & 7u;
    unsigned v;
    unsigned long long w;
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"((unsigned)(uintptr_t)(b + off)));
    asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(w) : "v"((unsigned)(uintptr_t)(b + off)));
    const unsigned w0 = (unsigned)w, w1 = (unsigned)(w >> 32);
    if (threadIdx.x < 8) { out[3 * threadIdx.x] = v; out[3 * threadIdx.x + 1] = w0; out[3 * threadIdx.x + 2] = w1; }
}

template <int MIS>
__global__ void __launch_bounds__(256) k_time(unsigned *out, unsigned stride) {
    __shared__ unsigned char b[16384];
    for (int i = threadIdx.x; i < 16384; i += 256) b[i] = (unsigned char)i;
    __syncthreads();
    unsigned acc = 0;
    unsigned a = (threadIdx.x * stride + MIS) & 8191u;
    for (int i = 0; i < 4096; ++i) {
        unsigned v;
        asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"((unsigned)(uintptr_t)(b + a)));
        acc += v;
        a = (a + 36u) & 8191u;
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

int main() {
    unsigned *d, h[24];
    if (hipMalloc(&d, 1 << 22) != hipSuccess) return 1;
    hipLaunchKernelGGL(k_check, dim3(1), dim3(64), 0, 0, d);
    if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    printf("{\"reads\": [");
    for (int i = 0; i < 8; ++i) printf("%s{\"off\": %d, \"b32\": \"0x%08x\", \"b64\": \"0x%08x%08x\"}", i ? ", " : "", i, h[3 * i], h[3 * i + 2], h[3 * i + 1]);
    printf("],\n");
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float ms[2];
    for (int m = 0; m < 2; ++m) {
        for (int r = 0; r < 2; ++r) {
            (void)hipEventRecord(e0, 0);
            if (m == 0) hipLaunchKernelGGL(k_time<0>, dim3(1024), dim3(256), 0, 0, d, 36u);
            else hipLaunchKernelGGL(k_time<1>, dim3(1024), dim3(256), 0, 0, d, 36u);
            (void)hipEventRecord(e1, 0);
            (void)hipEventSynchronize(e1);
            (void)hipEventElapsedTime(&ms[m], e0, e1);
        }
    }
    printf(" \"aligned_ms\": %.3f, \"unaligned_ms\": %.3f}\n", ms[0], ms[1]);
    return 0;
}
