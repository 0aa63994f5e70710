// Probe: issue cost per wave64 instruction on one gfx950 SIMD, by instruction and by waves per SIMD.
// Every wave runs 8 independent chains of one instruction (inline asm, 512 iterations); s_memtime
// around the loop gives shader cycles per wave; cycles per instruction per SIMD =
// wave cycles / (instructions per wave * waves per SIMD). One workgroup of 4 x W waves per CU.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probe/issue_rate tools/probe/issue_rate.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int kIter = 512, kChains = 8;

#define OP8(INSN, CON)                                                                                   \
    asm volatile(INSN : "+v"(a[0]) : CON(b)); asm volatile(INSN : "+v"(a[1]) : CON(b));                 \
    asm volatile(INSN : "+v"(a[2]) : CON(b)); asm volatile(INSN : "+v"(a[3]) : CON(b));                 \
    asm volatile(INSN : "+v"(a[4]) : CON(b)); asm volatile(INSN : "+v"(a[5]) : CON(b));                 \
    asm volatile(INSN : "+v"(a[6]) : CON(b)); asm volatile(INSN : "+v"(a[7]) : CON(b));

template <int OP>
__global__ void k_probe(uint32_t seed, unsigned long long* cyc, uint32_t* sink) {
    uint32_t a[kChains];
    for (int i = 0; i < kChains; ++i) a[i] = seed * (i + 3) + threadIdx.x;
    uint32_t b = seed ^ threadIdx.x;
    uint32_t s0 = seed, s1 = seed + 1, s2 = seed + 2, s3 = seed + 3;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < kIter; ++it) {
        if constexpr (OP == 0) { OP8("v_add_u32 %0, %0, %1", "v") }
        else if constexpr (OP == 1) { OP8("v_alignbyte_b32 %0, %0, %1, 3", "v") }
        else if constexpr (OP == 2) { OP8("v_ffbl_b32 %0, %0", "v") }
        else if constexpr (OP == 3) { OP8("v_mul_lo_u32 %0, %0, %1", "v") }
        else if constexpr (OP == 4) { OP8("v_xor_b32 %0, %0, %1", "v") }
        else if constexpr (OP == 5) { OP8("v_min_u32 %0, %0, %1", "v") }
        else if constexpr (OP == 6) { OP8("v_lshl_add_u32 %0, %0, 3, %1", "v") }
        else if constexpr (OP == 7) {  // SALU chains
            asm volatile("s_add_u32 %0, %0, 7" : "+s"(s0)); asm volatile("s_add_u32 %0, %0, 7" : "+s"(s1));
            asm volatile("s_add_u32 %0, %0, 7" : "+s"(s2)); asm volatile("s_add_u32 %0, %0, 7" : "+s"(s3));
            asm volatile("s_add_u32 %0, %0, 7" : "+s"(s0)); asm volatile("s_add_u32 %0, %0, 7" : "+s"(s1));
            asm volatile("s_add_u32 %0, %0, 7" : "+s"(s2)); asm volatile("s_add_u32 %0, %0, 7" : "+s"(s3));
        } else if constexpr (OP == 8) {  // VALU and SALU interleaved 1:1
            asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[0]) : "v"(b)); asm volatile("s_add_u32 %0, %0, 7" : "+s"(s0));
            asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[1]) : "v"(b)); asm volatile("s_add_u32 %0, %0, 7" : "+s"(s1));
            asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[2]) : "v"(b)); asm volatile("s_add_u32 %0, %0, 7" : "+s"(s2));
            asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[3]) : "v"(b)); asm volatile("s_add_u32 %0, %0, 7" : "+s"(s3));
            asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[4]) : "v"(b)); asm volatile("s_add_u32 %0, %0, 7" : "+s"(s0));
            asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[5]) : "v"(b)); asm volatile("s_add_u32 %0, %0, 7" : "+s"(s1));
            asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[6]) : "v"(b)); asm volatile("s_add_u32 %0, %0, 7" : "+s"(s2));
            asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[7]) : "v"(b)); asm volatile("s_add_u32 %0, %0, 7" : "+s"(s3));
        } else if constexpr (OP == 9) {  // v_cndmask with vcc
            asm volatile("v_cmp_gt_u32 vcc, %0, %1\n v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[0]) : "v"(b) : "vcc");
            asm volatile("v_cmp_gt_u32 vcc, %0, %1\n v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[1]) : "v"(b) : "vcc");
            asm volatile("v_cmp_gt_u32 vcc, %0, %1\n v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[2]) : "v"(b) : "vcc");
            asm volatile("v_cmp_gt_u32 vcc, %0, %1\n v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[3]) : "v"(b) : "vcc");
        } else if constexpr (OP == 10) {  // ds_read_b32 at distinct banks (throughput, conflict-free)
            __shared__ uint32_t lds[4096];
            a[0] += lds[(threadIdx.x + a[0]) & 63]; a[1] += lds[((threadIdx.x + a[1]) & 63) + 64];
            a[2] += lds[((threadIdx.x + a[2]) & 63) + 128]; a[3] += lds[((threadIdx.x + a[3]) & 63) + 192];
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    uint32_t r = s0 ^ s1 ^ s2 ^ s3;
    for (int i = 0; i < kChains; ++i) r ^= a[i];
    if (r == 0x12345678u) sink[threadIdx.x] = r;
    if ((threadIdx.x & 63) == 0) atomicAdd(cyc, t1 - t0);
}

template <int OP>
static void run(const char* name, int instr_per_iter, unsigned long long* d, uint32_t* sink) {
    for (int W = 1; W <= 4; W *= 2) {
        hipMemset(d, 0, 8);
        const int threads = 256 * W;  // 4 SIMDs x W waves
        hipLaunchKernelGGL(k_probe<OP>, dim3(256), dim3(threads), 0, 0, 1u, d, sink);
        hipError_t e = hipDeviceSynchronize();
        if (e != hipSuccess) { printf("%s W=%d: %s\n", name, W, hipGetErrorString(e)); fflush(stdout); return; }
        unsigned long long c = 0;
        hipMemcpy(&c, d, 8, hipMemcpyDeviceToHost);
        const double waves = 256.0 * 4 * W;
        const double per_wave = (double)c / waves;
        printf("%-22s W=%d  wave cycles %8.0f  cycles/instr/SIMD %.2f\n", name, W, per_wave,
               per_wave / ((double)kIter * instr_per_iter * W));
        fflush(stdout);
    }
}

int main() {
    setvbuf(stdout, nullptr, _IONBF, 0);
    printf("start\n");
    unsigned long long* d;
    uint32_t* sink;
    hipMalloc(&d, 8);
    hipMalloc(&sink, 4096 * 4);
    run<0>("v_add_u32", 8, d, sink);
    run<1>("v_alignbyte_b32", 8, d, sink);
    run<2>("v_ffbl_b32", 8, d, sink);
    run<3>("v_mul_lo_u32", 8, d, sink);
    run<4>("v_xor_b32", 8, d, sink);
    run<5>("v_min_u32", 8, d, sink);
    run<6>("v_lshl_add_u32", 8, d, sink);
    run<7>("s_add_u32", 8, d, sink);
    run<8>("v_add+s_add (16)", 16, d, sink);
    run<9>("v_cmp+v_cndmask (8)", 8, d, sink);
    run<10>("ds_read_b32+v_add (8)", 8, d, sink);
    return 0;
}
