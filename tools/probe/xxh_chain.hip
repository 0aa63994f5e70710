// Probe: how fast can xxh32's serial stripe chain run on gfx950?
// acc' = rotl(acc + m * P2, 13) * P1 per 16-byte stripe (4 independent accumulators). 1 MiB,
// inputs prefetched well ahead, timed with events; results checked against the host.
//   v0: k_dframe_close's form: lanes 4k..4k+3 own accumulators 0..3 of one range, each lane loads
//       its own dwords (32 in flight), chain add -> rotate -> multiply, multiply by P2 per stripe
//   v1: as v0, with the P2 multiply and the add fused (v_mad_u64_u32)
//   v2: one range per wave: lane 4k + a loads stripe k's dword a and multiplies it by P2 (one
//       load and one multiply per 16 stripes), the values reach accumulator a by ds_bpermute
//   v3: four waves, one accumulator each on the scalar unit (five SALU instructions per round)
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probe/xxh_chain tools/probe/xxh_chain.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

constexpr uint32_t P1 = 2654435761U, P2 = 2246822519U;
__device__ __forceinline__ uint32_t rotl13(uint32_t x) { return __builtin_amdgcn_alignbit(x, x, 19); }

constexpr uint32_t kIF = 32;  // stripes per batch (loads in flight per lane)

template <int V>
__global__ __launch_bounds__(64) void k_lanes(const uint32_t* __restrict__ in, uint32_t nstripes, uint32_t* out) {
    const uint32_t a = threadIdx.x & 3;
    uint32_t acc = a == 0 ? P1 + P2 : (a == 1 ? P2 : (a == 2 ? 0u : 0u - P1));
    const uint32_t* w = in + a;
    for (uint32_t s = 0; s < nstripes; s += kIF) {
        uint32_t v[kIF];
#pragma unroll
        for (uint32_t k = 0; k < kIF; ++k) v[k] = w[4 * (s + k)];
#pragma unroll
        for (uint32_t k = 0; k < kIF; ++k) {
            if constexpr (V == 0) acc = rotl13(acc + v[k] * P2) * P1;
            else acc = rotl13((uint32_t)((uint64_t)v[k] * P2 + acc)) * P1;
        }
    }
    if (threadIdx.x < 4) out[threadIdx.x] = acc;
}

constexpr int kAhead = 8;  // batches of 16 stripes in flight (v2)
__global__ __launch_bounds__(64) void k_wave(const uint32_t* __restrict__ in, uint32_t nstripes, uint32_t* out) {
    const int lane = threadIdx.x;
    const uint32_t a = lane & 3;
    uint32_t acc = a == 0 ? P1 + P2 : (a == 1 ? P2 : (a == 2 ? 0u : 0u - P1));
    const uint32_t nb = nstripes / 16;
    uint32_t q[kAhead];
#pragma unroll
    for (int k = 0; k < kAhead; ++k) q[k] = (uint32_t)k < nb ? in[k * 64 + lane] : 0u;
    for (uint32_t b = 0; b < nb; b += kAhead) {
#pragma unroll
        for (int u = 0; u < kAhead; ++u) {
            const uint32_t cur = q[u] * P2;
            if (b + kAhead + u < nb) q[u] = in[(b + kAhead + u) * 64 + lane];
            uint32_t m[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) m[k] = __builtin_amdgcn_ds_bpermute((4 * k + (int)a) << 2, (int)cur);
#pragma unroll
            for (int k = 0; k < 16; ++k) acc = rotl13(acc + m[k]) * P1;
        }
    }
    if (lane < 4) out[lane] = acc;
}

__device__ __forceinline__ uint32_t salu_round(uint32_t acc, uint32_t mp) {
    uint32_t y, t;
    asm volatile(
        "s_add_u32 %0, %2, %3\n\t"
        "s_lshl_b32 %1, %0, 13\n\t"
        "s_lshr_b32 %0, %0, 19\n\t"
        "s_or_b32 %0, %0, %1\n\t"
        "s_mul_i32 %0, %0, %4\n\t"
        : "=&s"(y), "=&s"(t)
        : "s"(acc), "s"(mp), "s"(P1)
        : "scc");
    return y;
}
__global__ __launch_bounds__(256) void k_salu(const uint32_t* __restrict__ in, uint32_t nstripes, uint32_t* out) {
    const uint32_t a = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint32_t acc = __builtin_amdgcn_readfirstlane(a == 0 ? P1 + P2 : (a == 1 ? P2 : (a == 2 ? 0u : 0u - P1)));
    const uint32_t* p = in + a;
    for (uint32_t s = 0; s < nstripes; s += 16) {
        uint32_t m[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) m[k] = __builtin_amdgcn_readfirstlane(p[4 * (s + k)]) * P2;
#pragma unroll
        for (int k = 0; k < 16; ++k) acc = salu_round(acc, m[k]);
    }
    if ((threadIdx.x & 63) == 0) out[a] = acc;
}

static uint32_t rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

int main() {
    const uint32_t bytes = 1u << 20, ns = bytes / 16;
    uint32_t* h = (uint32_t*)malloc(bytes);
    for (uint32_t i = 0; i < bytes / 4; ++i) h[i] = i * 2654435761u ^ (i >> 3);
    uint32_t ref[4] = {P1 + P2, P2, 0, 0u - P1};
    for (uint32_t s = 0; s < ns; ++s)
        for (int a = 0; a < 4; ++a) ref[a] = rotl(ref[a] + h[4 * s + a] * P2, 13) * P1;
    uint32_t *d, *o;
    (void)hipMalloc(&d, bytes + 4096);
    (void)hipMalloc(&o, 64);
    (void)hipMemcpy(d, h, bytes, hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int v = 0; v < 4; ++v) {
        float best = 1e9;
        for (int rep = 0; rep < 5; ++rep) {
            (void)hipMemset(o, 0, 64);
            (void)hipEventRecord(e0);
            if (v == 0) hipLaunchKernelGGL(k_lanes<0>, 1, 64, 0, 0, d, ns, o);
            if (v == 1) hipLaunchKernelGGL(k_lanes<1>, 1, 64, 0, 0, d, ns, o);
            if (v == 2) hipLaunchKernelGGL(k_wave, 1, 64, 0, 0, d, ns, o);
            if (v == 3) hipLaunchKernelGGL(k_salu, 1, 256, 0, 0, d, ns, o);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            if (ms < best) best = ms;
        }
        uint32_t got[4];
        (void)hipMemcpy(got, o, 16, hipMemcpyDeviceToHost);
        const bool ok = memcmp(got, ref, 16) == 0;
        printf("{\"variant\": %d, \"ms_per_MiB\": %.4f, \"cycles_per_stripe_at_2.4GHz\": %.1f, \"ok\": %s}\n", v, best,
               best * 1e-3 * 2.4e9 / ns, ok ? "true" : "false");
    }
    return 0;
}
