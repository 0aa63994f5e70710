// Probe: do unaligned LDS loads (ds_read_b32 / b64 / b128 at any byte offset) return the bytes at
// that offset on this GPU? Prints OK / MISMATCH counts. Standalone diagnostic, not product code.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
typedef uint32_t u32u __attribute__((aligned(1)));
typedef uint64_t u64u __attribute__((aligned(1)));
typedef uint4 u128u __attribute__((aligned(1)));
__global__ void k(const uint8_t* g, uint32_t* o32, uint64_t* o64, uint4* o128) {
    __shared__ uint8_t s[8192];
    for (int i = threadIdx.x; i < 8192; i += blockDim.x) s[i] = g[i];
    __syncthreads();
    const uint32_t off = threadIdx.x * 7 + blockIdx.x;  // every byte phase
    o32[blockIdx.x * 256 + threadIdx.x] = *(const u32u*)(s + off);
    o64[blockIdx.x * 256 + threadIdx.x] = *(const u64u*)(s + off);
    o128[blockIdx.x * 256 + threadIdx.x] = *(const u128u*)(s + off);
}
int main() {
    const int nb = 16, nt = 256;
    uint8_t h[8192];
    for (int i = 0; i < 8192; ++i) h[i] = (uint8_t)(i * 131 + (i >> 8) * 7 + 1);
    uint8_t* dg; uint32_t* d32; uint64_t* d64; uint4* d128;
    hipMalloc(&dg, 8192); hipMalloc(&d32, nb * nt * 4); hipMalloc(&d64, nb * nt * 8); hipMalloc(&d128, nb * nt * 16);
    hipMemcpy(dg, h, 8192, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(nb), dim3(nt), 0, 0, dg, d32, d64, d128);
    uint32_t r32[nb * nt]; uint64_t r64[nb * nt]; uint4 r128[nb * nt];
    hipMemcpy(r32, d32, sizeof r32, hipMemcpyDeviceToHost);
    hipMemcpy(r64, d64, sizeof r64, hipMemcpyDeviceToHost);
    hipMemcpy(r128, d128, sizeof r128, hipMemcpyDeviceToHost);
    int bad32 = 0, bad64 = 0, bad128 = 0;
    for (int b = 0; b < nb; ++b)
        for (int t = 0; t < nt; ++t) {
            const int off = t * 7 + b, i = b * nt + t;
            uint32_t e32; uint64_t e64; uint4 e128;
            __builtin_memcpy(&e32, h + off, 4); __builtin_memcpy(&e64, h + off, 8); __builtin_memcpy(&e128, h + off, 16);
            bad32 += r32[i] != e32; bad64 += r64[i] != e64;
            bad128 += r128[i].x != e128.x || r128[i].y != e128.y || r128[i].z != e128.z || r128[i].w != e128.w;
        }
    printf("unaligned LDS reads: b32 %s (%d bad), b64 %s (%d bad), b128 %s (%d bad) of %d\n", bad32 ? "MISMATCH" : "OK",
           bad32, bad64 ? "MISMATCH" : "OK", bad64, bad128 ? "MISMATCH" : "OK", bad128, nb * nt);
    return 0;
}
