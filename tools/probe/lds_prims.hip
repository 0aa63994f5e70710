// Probe: throughput and semantics of the LDS primitives a byte-scatter LZ4 executor could use
// on gfx950 — aligned vs misaligned ds_read/ds_write b32/b128, ds_write_b8, atomic ds_or_b32,
// ds_mskor_b32 — and misaligned global_load_dwordx4. Standalone diagnostic, not product code.
// Prints, per primitive: correctness (where checkable) and cycles per wave-instruction per CU.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef uint32_t v2u __attribute__((ext_vector_type(2)));
#define ITERS 256
#define UNR 16

enum Mode {
    RD32_AL, RD32_MIS, RD128_AL, RD128_MIS, RD128_MIS_RAND, WR32_AL, WR32_MIS, WR128_AL, WR128_MIS, WR8, OR32, MSKOR32,
    RDU8, WR64_MIS, NMODES
};
static const char* kName[] = {"ds_read_b32 aligned", "ds_read_b32 misaligned(+1)", "ds_read_b128 aligned",
                              "ds_read_b128 misaligned(+1..15 by lane)", "ds_read_b128 misaligned random",
                              "ds_write_b32 aligned", "ds_write_b32 misaligned(+1)", "ds_write_b128 aligned",
                              "ds_write_b128 misaligned(+lane%16)", "ds_write_b8", "ds_or_b32 (atomic)",
                              "ds_mskor_b32 (atomic)", "ds_read_u8", "ds_write_b64 misaligned"};

template <int M>
__global__ __launch_bounds__(256) void kprobe(uint32_t* sink, uint64_t* cyc) {
    __shared__ __attribute__((aligned(16))) uint8_t s[16384];
    const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
    for (uint32_t i = t; i < 16384 / 4; i += 256) ((uint32_t*)s)[i] = i * 2654435761u;
    __syncthreads();
    uint32_t base = w * 4096;  // each wave its own 4 KiB
    uint32_t addr;
    if (M == RD32_MIS || M == WR32_MIS) addr = base + lane * 4 + 1;
    else if (M == RD128_AL || M == WR128_AL) addr = base + lane * 16;
    else if (M == RD128_MIS || M == WR128_MIS) addr = base + lane * 16 + 1 + (lane & 7) * 2 % 15;
    else if (M == RD128_MIS_RAND) addr = base + ((lane * 2654435761u) >> 20) % 4000;
    else if (M == WR64_MIS) addr = base + lane * 8 + 3;
    else if (M == WR8 || M == RDU8) addr = base + lane * 3;
    else addr = base + lane * 4;
    uint32_t acc = 0;
    v4u v4 = {lane, lane + 1, lane + 2, lane + 3};
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            if (M == RD32_AL || M == RD32_MIS) {
                uint32_t x;
                asm volatile("ds_read_b32 %0, %1" : "=v"(x) : "v"(addr));
                acc += x;
            } else if (M == RDU8) {
                uint32_t x;
                asm volatile("ds_read_u8 %0, %1" : "=v"(x) : "v"(addr));
                acc += x;
            } else if (M == RD128_AL || M == RD128_MIS || M == RD128_MIS_RAND) {
                v4u x;
                asm volatile("ds_read_b128 %0, %1" : "=v"(x) : "v"(addr));
                acc += x.x ^ x.w;
            } else if (M == WR32_AL || M == WR32_MIS) {
                asm volatile("ds_write_b32 %0, %1" ::"v"(addr), "v"(acc + u));
            } else if (M == WR128_AL || M == WR128_MIS) {
                asm volatile("ds_write_b128 %0, %1" ::"v"(addr), "v"(v4));
            } else if (M == WR64_MIS) {
                v2u v2 = {v4.x, v4.y};
                asm volatile("ds_write_b64 %0, %1" ::"v"(addr), "v"(v2));
            } else if (M == WR8) {
                asm volatile("ds_write_b8 %0, %1" ::"v"(addr), "v"(acc + u));
            } else if (M == OR32) {
                asm volatile("ds_or_b32 %0, %1" ::"v"(addr), "v"(acc + u));
            } else if (M == MSKOR32) {
                asm volatile("ds_mskor_b32 %0, %1, %2" ::"v"(addr), "v"(0xFF00FF00u), "v"(acc + u));
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    __syncthreads();
    if (lane == 0) cyc[blockIdx.x * 4 + w] = t1 - t0;
    sink[blockIdx.x * 256 + t] = acc;
}

// misaligned write semantics: wave writes 16 bytes at byte offsets; check the image
__global__ void ksem(uint8_t* out) {
    __shared__ __attribute__((aligned(16))) uint8_t s[4096];
    const uint32_t t = threadIdx.x;
    for (uint32_t i = t; i < 4096; i += 64) s[i] = 0xEE;
    __syncthreads();
    // lane t writes 16 bytes at 40*t + (t % 16) (regions disjoint)
    const uint32_t a = 40 * t + (t % 16);
    v4u v;
    for (int k = 0; k < 4; ++k) { uint32_t x = 0; for (int j = 0; j < 4; ++j) x |= (uint32_t)(uint8_t)(t * 16 + 4 * k + j) << (8 * j); v[k] = x; }
    asm volatile("ds_write_b128 %0, %1" ::"v"(a), "v"(v));
    // and 4 bytes at 40*t + 30 + (t%4) with ds_write_b32, 8 at 40*t+20+(t%8)... keep simple: b32
    uint32_t v32 = 0xA0B0C0D0u + t;
    asm volatile("ds_write_b32 %0, %1" ::"v"(40 * t + 33 + (t % 3)), "v"(v32));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
    for (uint32_t i = t; i < 4096; i += 64) out[i] = s[i];
}

// ds_mskor semantics: MEM = (MEM & ~DATA) | DATA2
__global__ void kmsk(uint32_t* out) {
    __shared__ uint32_t s[64];
    const uint32_t t = threadIdx.x;
    s[t] = 0x11223344u;
    __syncthreads();
    asm volatile("ds_mskor_b32 %0, %1, %2" ::"v"(t * 4), "v"(0x0000FF00u), "v"(0x0000AB00u));
    // two lanes hitting the same dword with disjoint bytes in one instruction
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const uint32_t d = (t / 2) * 4;
    const uint32_t m = (t & 1) ? 0xFF000000u : 0x000000FFu;
    asm volatile("ds_mskor_b32 %0, %1, %2" ::"v"(d), "v"(m), "v"((t & 1) ? 0x77000000u : 0x00000066u));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
    out[t] = s[t];
}

// misaligned global loads
__global__ void kglob(const uint8_t* g, uint4* o, uint64_t* cyc, int mis) {
    const uint32_t t = threadIdx.x + blockIdx.x * blockDim.x;
    const uint8_t* p = g + (size_t)t * 16 + (mis ? (t % 15) + 1 : 0);
    typedef uint4 u128u __attribute__((aligned(1)));
    uint4 acc = make_uint4(0, 0, 0, 0);
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < 64; ++i) {
        uint4 x = *(const u128u*)(p + (size_t)i * 262144 * 16);
        acc.x ^= x.x; acc.y += x.y; acc.z ^= x.z; acc.w += x.w;
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    o[t] = acc;
    if ((threadIdx.x & 63) == 0) cyc[t / 64] = t1 - t0;
}

template <int M>
static void run(int blocks, uint32_t* sink, uint64_t* dcyc, uint64_t* hcyc) {
    hipLaunchKernelGGL(kprobe<M>, dim3(blocks), dim3(256), 0, 0, sink, dcyc);
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    hipEventRecord(a);
    hipLaunchKernelGGL(kprobe<M>, dim3(blocks), dim3(256), 0, 0, sink, dcyc);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    hipMemcpy(hcyc, dcyc, blocks * 4 * 8, hipMemcpyDeviceToHost);
    double mx = 0, avg = 0;
    for (int i = 0; i < blocks * 4; ++i) { mx = hcyc[i] > mx ? hcyc[i] : mx; avg += hcyc[i]; }
    avg /= blocks * 4;
    const double insts_per_wave = (double)ITERS * UNR;
    const int per_cu = blocks / 256 * 4;  // waves per CU
    // per-CU cycles per wave-instruction: wave span / (instructions of all waves on the CU)
    printf("%-40s waves/CU %2d  wave span %8.0f cyc  -> %6.2f cyc per wave-instr per CU  (%.3f ms)\n", kName[M],
           per_cu, avg, avg / (insts_per_wave * per_cu), ms);
}

int main() {
    uint32_t* sink; uint64_t* dcyc;
    hipMalloc(&sink, 2048 * 256 * 4);
    hipMalloc(&dcyc, 2048 * 4 * 8);
    static uint64_t hcyc[2048 * 4];
    for (int blocks : {256, 1024, 2048}) {
        run<RD32_AL>(blocks, sink, dcyc, hcyc);
        run<RD32_MIS>(blocks, sink, dcyc, hcyc);
        run<RDU8>(blocks, sink, dcyc, hcyc);
        run<RD128_AL>(blocks, sink, dcyc, hcyc);
        run<RD128_MIS>(blocks, sink, dcyc, hcyc);
        run<RD128_MIS_RAND>(blocks, sink, dcyc, hcyc);
        run<WR32_AL>(blocks, sink, dcyc, hcyc);
        run<WR32_MIS>(blocks, sink, dcyc, hcyc);
        run<WR64_MIS>(blocks, sink, dcyc, hcyc);
        run<WR128_AL>(blocks, sink, dcyc, hcyc);
        run<WR128_MIS>(blocks, sink, dcyc, hcyc);
        run<WR8>(blocks, sink, dcyc, hcyc);
        run<OR32>(blocks, sink, dcyc, hcyc);
        run<MSKOR32>(blocks, sink, dcyc, hcyc);
    }
    // semantics
    uint8_t* dout; hipMalloc(&dout, 4096);
    hipLaunchKernelGGL(ksem, dim3(1), dim3(64), 0, 0, dout);
    static uint8_t img[4096];
    hipMemcpy(img, dout, 4096, hipMemcpyDeviceToHost);
    static uint8_t exp_[4096];
    memset(exp_, 0xEE, sizeof exp_);
    for (int t = 0; t < 64; ++t) {
        const int a = 40 * t + (t % 16);
        for (int k = 0; k < 16; ++k) exp_[a + k] = (uint8_t)(t * 16 + k);
        uint32_t v32 = 0xA0B0C0D0u + t;
        memcpy(exp_ + 40 * t + 33 + (t % 3), &v32, 4);
    }
    int bad = 0;
    for (int i = 0; i < 4096; ++i) bad += img[i] != exp_[i];
    printf("misaligned ds_write_b128/b32 image: %s (%d bad bytes)\n", bad ? "MISMATCH" : "OK", bad);
    uint32_t* dm; hipMalloc(&dm, 256);
    hipLaunchKernelGGL(kmsk, dim3(1), dim3(64), 0, 0, dm);
    uint32_t hm[64];
    hipMemcpy(hm, dm, 256, hipMemcpyDeviceToHost);
    int mbad = 0;
    for (int t = 0; t < 64; ++t) {
        uint32_t e = (0x11223344u & ~0x0000FF00u) | 0x0000AB00u;
        if (t < 32) e = (e & 0x00FFFF00u) | 0x77000066u;
        mbad += hm[t] != e;
    }
    printf("ds_mskor_b32 semantics (incl. two lanes per dword): %s (%d bad) e.g. %08x\n", mbad ? "MISMATCH" : "OK", mbad, hm[0]);
    // global
    uint8_t* g; uint4* o; uint64_t* gc;
    const size_t gsz = (size_t)64 * 262144 * 16 + 4096;
    hipMalloc(&g, gsz); hipMalloc(&o, 262144 * 16); hipMalloc(&gc, 4096 * 8);
    hipMemset(g, 1, gsz);
    for (int mis = 0; mis < 2; ++mis) {
        hipLaunchKernelGGL(kglob, dim3(1024), dim3(256), 0, 0, g, o, gc, mis);
        hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
        hipEventRecord(a);
        hipLaunchKernelGGL(kglob, dim3(1024), dim3(256), 0, 0, g, o, gc, mis);
        hipEventRecord(b); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        printf("global_load_dwordx4 %s: %.3f ms for %.0f MB -> %.1f GB/s\n", mis ? "misaligned" : "aligned", ms,
               64.0 * 262144 * 16 / 1e6, 64.0 * 262144 * 16 / (ms * 1e6));
    }
    return 0;
}
