// Probe: does an unaligned LDS store (ds_write_b32 at any byte offset, what an aligned(1) u32
// store compiles to on gfx950) write exactly its 4 bytes there? Prints OK / MISMATCH counts.
// Standalone diagnostic, not product code.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
typedef uint32_t u32u __attribute__((aligned(1)));
__global__ void k(uint8_t* o) {
    __shared__ uint8_t s[4096];
    for (int i = threadIdx.x; i < 4096; i += blockDim.x) s[i] = 0xA5;
    __syncthreads();
    const uint32_t off = threadIdx.x * 5 + blockIdx.x;  // disjoint 4-byte ranges, every byte phase
    *(u32u*)(s + off) = 0x01020304u * (threadIdx.x + 1) ^ blockIdx.x;
    __syncthreads();
    for (int i = threadIdx.x; i < 4096; i += blockDim.x) o[blockIdx.x * 4096 + i] = s[i];
}
int main() {
    const int nb = 8, nt = 256;
    uint8_t* d;
    hipMalloc(&d, nb * 4096);
    hipLaunchKernelGGL(k, dim3(nb), dim3(nt), 0, 0, d);
    static uint8_t h[nb * 4096];
    hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int b = 0; b < nb; ++b) {
        uint8_t e[4096];
        for (int i = 0; i < 4096; ++i) e[i] = 0xA5;
        for (int t = 0; t < nt; ++t) {
            const uint32_t v = 0x01020304u * (t + 1) ^ b;
            __builtin_memcpy(e + t * 5 + b, &v, 4);
        }
        for (int i = 0; i < 4096; ++i) bad += h[b * 4096 + i] != e[i];
    }
    printf("unaligned LDS b32 stores: %s (%d bad bytes of %d)\n", bad ? "MISMATCH" : "OK", bad, nb * 4096);
    return 0;
}
