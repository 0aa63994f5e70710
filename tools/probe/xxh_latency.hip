// Probe: dependent latency of one xxh32 stripe round on gfx950 (one wave per SIMD, values in
// registers, s_memtime around 4096 rounds), by formulation:
//   v0: acc = rotl(acc + m * P2, 13) * P1 as the compiler emits it from C (m * P2 fused with the add)
//   v1: the product m * P2 precomputed off the chain: add -> v_alignbit -> v_mul_lo_u32 (inline asm)
//   v2: as v1 with the rotate as v_lshlrev + v_lshrrev + v_or (no alignbit)
//   v3: the bare chain of v_mul_lo_u32 alone (its latency)
//   v4: the bare chain of v_alignbit alone
//   v5: the bare chain of v_add_u32 alone
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probe/xxh_latency tools/probe/xxh_latency.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr uint32_t P1 = 2654435761U, P2 = 2246822519U;
constexpr int kR = 4096;

template <int V>
__global__ __launch_bounds__(64) void k_lat(const uint32_t* __restrict__ in, unsigned long long* cyc, uint32_t* out) {
    uint32_t acc = in[threadIdx.x];
    uint32_t m[16];
    for (int k = 0; k < 16; ++k) m[k] = in[64 + 16 * threadIdx.x + k];
    uint32_t p[16];
    for (int k = 0; k < 16; ++k) p[k] = m[k] * P2;
    const uint32_t p1 = P1;
    __builtin_amdgcn_s_waitcnt(0);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < kR; r += 16) {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            if constexpr (V == 0) {
                const uint32_t x = acc + m[k] * P2;
                acc = __builtin_amdgcn_alignbit(x, x, 19) * P1;
            } else if constexpr (V == 1) {
                asm volatile("v_add_u32 %0, %0, %1\n v_alignbit_b32 %0, %0, %0, 19\n v_mul_lo_u32 %0, %0, %2"
                             : "+v"(acc) : "v"(p[k]), "v"(p1));
            } else if constexpr (V == 2) {
                uint32_t t;
                asm volatile("v_add_u32 %0, %0, %2\n v_lshrrev_b32 %1, 19, %0\n v_lshl_or_b32 %0, %0, 13, %1\n v_mul_lo_u32 %0, %0, %3"
                             : "+v"(acc), "=&v"(t) : "v"(p[k]), "v"(p1));
            } else if constexpr (V == 3) {
                asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(acc) : "v"(p[k]));
            } else if constexpr (V == 4) {
                asm volatile("v_alignbit_b32 %0, %0, %1, 19" : "+v"(acc) : "v"(p[k]));
            } else {
                asm volatile("v_add_u32 %0, %0, %1" : "+v"(acc) : "v"(p[k]));
            }
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 64 + threadIdx.x] = acc;
    if (threadIdx.x == 0) atomicAdd(cyc, t1 - t0);
}

template <int V>
static void run(const char* name, const uint32_t* d_in, unsigned long long* d_cyc, uint32_t* d_out) {
    hipMemset(d_cyc, 0, 8);
    hipLaunchKernelGGL(k_lat<V>, dim3(1024), dim3(64), 0, 0, d_in, d_cyc, d_out);  // one wave per SIMD
    const hipError_t e = hipDeviceSynchronize();
    if (e != hipSuccess) { printf("%s: %s\n", name, hipGetErrorString(e)); return; }
    unsigned long long c = 0;
    hipMemcpy(&c, d_cyc, 8, hipMemcpyDeviceToHost);
    printf("%-44s %.1f cycles per round\n", name, (double)c / 1024.0 / kR);
}

int main() {
    setvbuf(stdout, nullptr, _IONBF, 0);
    uint32_t* d_in;
    unsigned long long* d_cyc;
    uint32_t* d_out;
    hipMalloc(&d_in, 64 * 20 * 4);
    hipMemset(d_in, 7, 64 * 20 * 4);
    hipMalloc(&d_cyc, 8);
    hipMalloc(&d_out, 1024 * 64 * 4);
    run<0>("v0 compiler form (mad with m*P2)", d_in, d_cyc, d_out);
    run<1>("v1 precomputed product: add+alignbit+mul_lo", d_in, d_cyc, d_out);
    run<2>("v2 precomputed product: add+shr+lshl_or+mul", d_in, d_cyc, d_out);
    run<3>("v3 v_mul_lo_u32 chain", d_in, d_cyc, d_out);
    run<4>("v4 v_alignbit_b32 chain", d_in, d_cyc, d_out);
    run<5>("v5 v_add_u32 chain", d_in, d_cyc, d_out);
    return 0;
}
