// s3hc_lb.hip — large-block LZ4 decode on CDNA4 (gfx950): one block, many workgroups.
//
// The one-wave-per-block decoder (k_decode_units) is the right shape for 64 KiB blocks, of
// which a batch holds thousands. The reference's own cache files are different: flush_batch
// (disk_cache.rs:1820-1870) compresses ~1 MiB batches with lz4_flex BlockSize::Auto, i.e. one
// block of up to 4 MiB per frame (BD 0x70), and a GET of such a file hands the GPU a handful
// of large blocks. Decoding those with one wave each leaves the chip idle, so blocks whose
// frame allows more than 64 KiB go through this path instead (same results, same statuses):
//
//   k_lb_classify  (1 workgroup)  takes the eligible units (one independent compressed block,
//                  frame max block size > 64 KiB) up to the scratch caps; lays out chunks of
//                  kLbChunk compressed positions per block.
//   k_lb_gran      per chunk: first non-255 byte at or after each 64-byte granule (length
//                  extension runs are 255-runs; this makes every run length O(64) to find).
//   k_lbt_walk     per chunk: speculative token walks from every 32-position segment, merged
//                  where they meet; each segment's chain exit (doubling over segments) and the
//                  exits of the chunk's first 64 positions.
//   k_lbt_entry    per block, serial over chunks: the true chain's entry into each chunk.
//   k_lbt_mark     per chunk: the true chain from the entry through the walks' marks (= the
//                  block's real tokens), parsed one per thread into records; per-chunk sequence
//                  count and output bytes. (k_lb_exit / k_lb_entry / k_lb_mark: the rounds 1-5
//                  tokenizer by next-token tables and pointer doubling, S3HC_LB_TOKV2=0 builds.)
//   (scans)        global sequence index and output offset of each chunk.
//   k_lb_seq       per chunk: the sequence table (out, literal, ll, ml, offset) from the records
//                  and the lz4_flex bound checks in stream order (first failing sequence decides).
//   k_lb_fin       per block: size, status, first sequence.
//   k_lb_run       (launches of many blocks) one 1024-thread workgroup per block writes the
//                  output in 7.5 KiB steps: in each step every byte gets its value (literal, or a
//                  match source before the step: 64 KiB LDS ring of recent output) or a pointer
//                  to its source inside the step (overlapping copies folded into the first
//                  period), and the pointers are jumped in LDS until every byte is final; its
//                  16th wave hashes the finished steps beside the 15 decoding waves' LDS barrier.
//   k_lbw_*        (launches of few large blocks) spread execution: every 7.5 KiB tile of every
//                  block at once, chains across tiles resolved by global pointer jumping.
//
// All of it is integer byte work (no MFMA); every kernel is bound by memory latency or LDS.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>

#include "s3hc_lz4.h"
#include "s3hc_plan.hpp"
#include "s3hc_knobs.hpp"

namespace s3hc {
namespace lb {
constexpr uint32_t kT = 1024;                  // threads of a tokenizing workgroup
constexpr uint32_t kPer = kLbChunk / kT;       // positions per thread
constexpr uint32_t kLook = 2048;               // staged bytes past the chunk
constexpr uint32_t kStage = kLbChunk + kLook;  // staged bytes per chunk
constexpr uint32_t kGran = 64;                 // 255-run index granule
constexpr uint32_t kGpc = kLbChunk / kGran;    // granules per chunk
constexpr uint32_t kTokSlot = kLbTokSlot;       // token records per chunk (trec)
constexpr uint32_t END = 0xFFFFFFFEu;          // next-token value: last sequence
constexpr uint32_t BAD = 0xFFFFFFFFu;          // next-token value: malformed token
constexpr uint32_t NONE = 0xFFFFFFFFu;
constexpr uint32_t INF = 0xFFFFFFFFu;
constexpr uint32_t kXT = 960;                  // decoding threads of an executing workgroup (15 waves)
constexpr uint32_t kXWG = kXT + 64;            // + one hashing wave
constexpr uint32_t kXPer = kLbStep / kXT;      // output bytes per executing thread per step (8)
// stripes the hashing wave takes in each phase of a step, sized to what the decoding waves
// spend there (measured phase lengths): one step needs kLbStep / 16 = 480
#ifndef S3HC_LBH_CLASSIFY  // (diagnostic builds sweep these)
#define S3HC_LBH_CLASSIFY 120
#endif
#ifndef S3HC_LBH_STORES
#define S3HC_LBH_STORES 90
#endif
#ifndef S3HC_LBH_INSTALL
#define S3HC_LBH_INSTALL 60
#endif
#ifndef S3HC_LBH_ROUND
#define S3HC_LBH_ROUND 80
#endif
#ifndef S3HC_LBH_LAG  // the classify phase hashes only while the wave lags more than this (bytes)
#define S3HC_LBH_LAG 0
#endif
#ifndef S3HC_LB_HOPS
#define S3HC_LB_HOPS 2  // A/B (tools_hops_ab.sh): 1 MiB step loop 2.00 -> 1.85 ms, 256 frames 4.58 -> 4.47; 3 and 4 lose
#endif
#ifndef S3HC_LB_XHOPS
#define S3HC_LB_XHOPS 2  // A/B (tools_xhops_ab.sh): 256 reference frames 4.39 -> 4.25 ms; 3 loses
#endif
constexpr uint32_t kXHops = S3HC_LB_XHOPS;    // hops per doubling level in k_lb_exit / k_lb_mark
constexpr uint32_t kJumpHops = S3HC_LB_HOPS;  // pointer hops per jumping round of k_lb_run
constexpr uint32_t kHashClassify = S3HC_LBH_CLASSIFY, kHashStores = S3HC_LBH_STORES, kHashInstall = S3HC_LBH_INSTALL,
                   kHashRound = S3HC_LBH_ROUND, kHashLag = S3HC_LBH_LAG;
static_assert(kXPer * kXT == kLbStep, "step geometry");
constexpr uint32_t kRing = 65536;              // recent output kept in LDS (match sources)
constexpr uint32_t kMaxSeqS = kLbStep / 4 + 3; // sequences touching one step (all but the last have sl >= 4)
constexpr uint32_t FIN = 0xFFFFFFFFu;          // source pointer of a final byte
constexpr uint32_t VALF = 0x80000000u;         // k_lb_run pointer-array entry of a final byte: VALF | value
}  // namespace lb

#if defined(S3HC_DIAG_LEVEL) && S3HC_DIAG_LEVEL == 10
#define S3HC_LBPROF 1
// diagnostic builds: k_lb_run phase times (s_memtime sums of every workgroup's thread 0):
// 0 owners, 1 classify + literal loads, 2 ring/pointer stores, 3 next step's sequences,
// 4 chain jumping, 5 flush, 6 -, 7 steps, 8 jump rounds, 9 loop top
__device__ unsigned long long g_lbprof[32];  // 12..17: k_lb_mark phases (thread 0 of each chunk); walks:
// 12..15 k_lbt_walk phases, 16..19 k_lbt_mark phases, 20..23 per-chunk maxima of walk-2 hops, first-
// position walk hops, entry-path hops and walk-2 re-marking hops (summed over chunks), 24 chunks
#endif

namespace {

__device__ __forceinline__ int lane64() { return (int)(threadIdx.x & 63u); }

// DPP lane moves (row_shr inside 16-lane rows, then row_bcast:15 / :31; lanes without a source
// read 0): wave scans without the LDS round trip of __shfl's ds_bpermute
template <int CTRL, int ROWMASK>
__device__ __forceinline__ uint32_t lb_dpp(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROWMASK, 0xF, false);
}
template <int CTRL, int ROWMASK>
__device__ __forceinline__ uint64_t lb_dpp(uint64_t x) {
    return (uint64_t)lb_dpp<CTRL, ROWMASK>((uint32_t)(x >> 32)) << 32 | lb_dpp<CTRL, ROWMASK>((uint32_t)x);
}
template <typename T>
__device__ __forceinline__ T wave_incl_add(T x, int) {
    x += lb_dpp<0x111, 0xF>(x);
    x += lb_dpp<0x112, 0xF>(x);
    x += lb_dpp<0x114, 0xF>(x);
    x += lb_dpp<0x118, 0xF>(x);
    x += lb_dpp<0x142, 0xA>(x);
    x += lb_dpp<0x143, 0xC>(x);
    return x;
}
__device__ __forceinline__ uint32_t lb_umax(uint32_t a, uint32_t b) { return a > b ? a : b; }
__device__ __forceinline__ uint32_t umin32_lb(uint32_t a, uint32_t b) { return a < b ? a : b; }
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t x) {
    x = lb_umax(x, lb_dpp<0x111, 0xF>(x));
    x = lb_umax(x, lb_dpp<0x112, 0xF>(x));
    x = lb_umax(x, lb_dpp<0x114, 0xF>(x));
    x = lb_umax(x, lb_dpp<0x118, 0xF>(x));
    x = lb_umax(x, lb_dpp<0x142, 0xA>(x));
    x = lb_umax(x, lb_dpp<0x143, 0xC>(x));
    return x;
}
// Owner scan of a step (k_lb_run, k_lbw_init): thread t holds the 16-bit start marks of bytes
// 8t .. 8t+7 (0 = no sequence starts there); each byte's owner is the running max of the marks
// up to it. Every thread of the workgroup calls (one barrier); shm: 16 aligned words.
template <typename Bar>
__device__ __forceinline__ uint4 lb_owners_b(const uint4 m4, uint32_t* shm, Bar bar) {
    const uint32_t mw[4] = {m4.x, m4.y, m4.z, m4.w};
    uint32_t mx = 0;
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) mx = lb_umax(mx, lb_umax(mw[k] & 0xFFFFu, mw[k] >> 16));
    const uint32_t inc = wave_incl_max(mx);
    const uint32_t w = threadIdx.x >> 6;
    if ((threadIdx.x & 63u) == 63u) shm[w] = inc;
    bar();
    uint32_t cur = lb_dpp<0x138, 0xF>(inc);  // wave_shr:1: the max before this lane (lane 0: 0)
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {  // and before this wave
        const uint4 v = ((const uint4*)shm)[k];
        cur = lb_umax(cur, 4u * k < w ? v.x : 0u);
        cur = lb_umax(cur, 4u * k + 1u < w ? v.y : 0u);
        cur = lb_umax(cur, 4u * k + 2u < w ? v.z : 0u);
        cur = lb_umax(cur, 4u * k + 3u < w ? v.w : 0u);
    }
    uint32_t ow[4];
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
        const uint32_t lo = mw[k] & 0xFFFFu, hi = mw[k] >> 16;
        cur = lb_umax(cur, lo);
        const uint32_t o0 = cur;
        cur = lb_umax(cur, hi);
        ow[k] = o0 | (cur << 16);
    }
    return make_uint4(ow[0], ow[1], ow[2], ow[3]);
}
__device__ __forceinline__ uint4 lb_owners(const uint4 m4, uint32_t* shm) {
    return lb_owners_b(m4, shm, [] { __syncthreads(); });
}
// The same scan in two halves with a barrier between them supplied by the caller (k_lb_run runs
// them inside the previous step's jumping rounds): lb_own1 publishes the wave's maximum and
// returns it (inclusive, per lane), lb_own2 gives the owners.
__device__ __forceinline__ uint32_t lb_own1(const uint4 m4, uint32_t* shm) {
    const uint32_t mw[4] = {m4.x, m4.y, m4.z, m4.w};
    uint32_t mx = 0;
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) mx = lb_umax(mx, lb_umax(mw[k] & 0xFFFFu, mw[k] >> 16));
    const uint32_t inc = wave_incl_max(mx);
    if ((threadIdx.x & 63u) == 63u) shm[threadIdx.x >> 6] = inc;
    return inc;
}
__device__ __forceinline__ uint4 lb_own2(const uint4 m4, uint32_t inc, const uint32_t* shm) {
    const uint32_t mw[4] = {m4.x, m4.y, m4.z, m4.w};
    const uint32_t w = threadIdx.x >> 6;
    uint32_t cur = lb_dpp<0x138, 0xF>(inc);  // wave_shr:1: the max before this lane (lane 0: 0)
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {  // and before this wave
        const uint4 v = ((const uint4*)shm)[k];
        cur = lb_umax(cur, 4u * k < w ? v.x : 0u);
        cur = lb_umax(cur, 4u * k + 1u < w ? v.y : 0u);
        cur = lb_umax(cur, 4u * k + 2u < w ? v.z : 0u);
        cur = lb_umax(cur, 4u * k + 3u < w ? v.w : 0u);
    }
    uint32_t ow[4];
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
        const uint32_t lo = mw[k] & 0xFFFFu, hi = mw[k] >> 16;
        cur = lb_umax(cur, lo);
        const uint32_t o0 = cur;
        cur = lb_umax(cur, hi);
        ow[k] = o0 | (cur << 16);
    }
    return make_uint4(ow[0], ow[1], ow[2], ow[3]);
}

// Barrier of k_lb_run's decoding waves only (S3HC_LB_XBAR): an LDS arrival counter; the hashing
// wave of the workgroup never waits on it (s_barrier counts every wave of the workgroup). A
// wave's LDS operations complete in order; the fences keep the compiler's order. (The spin is
// bounded so that a wrong count cannot hang the GPU: it ends the wait, and the results would be
// wrong, not the machine.)
__device__ __forceinline__ void lb_xbar(uint32_t* ctr, uint32_t& tgt, uint32_t nw) {
    tgt += nw;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if ((threadIdx.x & 63u) == 0u) {
        __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        for (uint32_t n = 0; n < (1u << 26); ++n)
            if (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= tgt) break;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// Workgroup exclusive sum (every thread calls; sh holds one entry per wave).
template <typename T, int NW>
__device__ __forceinline__ T wg_excl_add(T v, T* sh, T& total) {
    const int lane = lane64(), w = (int)(threadIdx.x >> 6);
    const T inc = wave_incl_add(v, lane);
    if (lane == 63) sh[w] = inc;
    __syncthreads();
    T pre = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < NW; ++k) {
        const T s = sh[k];
        pre += k < w ? s : (T)0;
        tot += s;
    }
    __syncthreads();
    total = tot;
    return pre + inc - v;
}

// Stage block bytes [cs, cs + ns) into LDS (aligned dword loads; returns s with s[i] = byte cs+i).
__device__ __forceinline__ const uint8_t* lb_stage(const uint8_t* g, uint32_t cs, uint32_t ns, uint8_t* raw) {
    const uintptr_t a0 = (uintptr_t)(g + cs);
    const uint32_t mis = (uint32_t)(a0 & 3u);
    const uint32_t* aw = (const uint32_t*)(a0 - mis);
    const uint32_t nd = (mis + ns + 3u) >> 2;
    // four loads per thread in flight before the LDS stores (one HBM round trip per 16 KiB)
    for (uint32_t base = 0; base < nd; base += 4u * blockDim.x) {
        uint32_t x[4];
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) {
            const uint32_t d = base + threadIdx.x + k * blockDim.x;
            x[k] = d < nd ? aw[d] : 0u;
        }
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) {
            const uint32_t d = base + threadIdx.x + k * blockDim.x;
            if (d < nd) ((uint32_t*)raw)[d] = x[k];
        }
    }
    return raw + mis;
}

struct LbView {
    const uint8_t* g;    // block payload in HBM
    const uint8_t* s;    // staged bytes: s[p - cs] for p in [cs, cs + ns)
    const uint32_t* nzg; // granule index, chunk-major
    uint32_t cs, ns, C, chunk0, nch;
};

__device__ __forceinline__ uint32_t lb_byte(const LbView& v, uint32_t p) {
    const uint32_t r = p - v.cs;
    return r < v.ns ? (uint32_t)v.s[r] : (uint32_t)v.g[p];
}

// First position >= pos (pos <= C) whose byte is not 255, or C.
__device__ uint32_t lb_nz(const LbView& v, uint32_t pos) {
    using namespace lb;
    uint32_t gend = (pos / kGran + 1u) * kGran;
    if (gend > v.C) gend = v.C;
    for (uint32_t k = pos; k < gend; ++k)
        if (lb_byte(v, k) != 255u) return k;
    if (gend >= v.C) return v.C;
    const uint32_t g = gend / kGran;
    uint32_t c = g / kGpc;
    uint32_t val = v.nzg[(size_t)(v.chunk0 + c) * kGpc + (g % kGpc)];
    while (val == INF) {
        if (++c >= v.nch) return v.C;
        val = v.nzg[(size_t)(v.chunk0 + c) * kGpc];
    }
    return val;
}

// The sequence whose token is at p, parsed with the rules of the one-wave decoder's exact path
// (dec_block slow path, lz4_flex decompress order). nxt: next token position, END (the literal
// run ends the block: last sequence) or BAD; late = 1: the literal run was valid before BAD,
// 2: the whole sequence was valid but no token follows its match.
struct LbTok {
    uint32_t nxt, lit, ll, off, ml, late;
};
__device__ LbTok lb_token(const LbView& v, uint32_t p) {
    using namespace lb;
    LbTok T;
    T.lit = 0; T.ll = 0; T.off = 0; T.ml = 0; T.late = 0;
    const uint32_t C = v.C;
    const uint32_t t = lb_byte(v, p);
    uint32_t pos = p + 1u;
    uint64_t ll = t >> 4;
    if (ll == 15u) {
        const uint32_t q = lb_nz(v, pos);
        if (q >= C) { T.nxt = BAD; return T; }
        ll = 15ull + 255ull * (q - pos) + lb_byte(v, q);
        pos = q + 1u;
    }
    if (ll > (uint64_t)(C - pos)) { T.nxt = BAD; return T; }
    T.lit = pos;
    T.ll = (uint32_t)ll;
    pos += (uint32_t)ll;
    if (pos == C) { T.nxt = END; return T; }
    T.late = 1;
    if (C - pos < 2u) { T.nxt = BAD; return T; }
    T.off = lb_byte(v, pos) | (lb_byte(v, pos + 1u) << 8);
    pos += 2u;
    uint32_t ml = (t & 15u) + 4u;
    if ((t & 15u) == 15u) {
        const uint32_t q = lb_nz(v, pos);
        if (q >= C) { T.nxt = BAD; return T; }
        ml = 19u + 255u * (q - pos) + lb_byte(v, q);  // q - pos < C <= 4 MiB: no overflow
        pos = q + 1u;
    }
    T.ml = ml;
    if (pos >= C) {  // a token must follow a match: the sequence itself is complete (late = 2)
        T.nxt = BAD;
        T.late = 2;
        return T;
    }
    T.late = 0;
    T.nxt = pos;
    return T;
}

// lb_token(v, p).nxt without reading the offset: the token (and one literal-length byte), then
// the match-length byte after the offset; length runs with a 255 byte take lb_token.
__device__ __forceinline__ uint32_t lb_next(const LbView& v, uint32_t p) {
    using namespace lb;
    const uint32_t C = v.C;
    const uint32_t t = lb_byte(v, p);
    const uint32_t L = t >> 4;
    uint32_t pos, ll;
    if (L < 15u) {
        ll = L;
        pos = p + 1u;
    } else {
        const uint32_t e1 = p + 1u < C ? lb_byte(v, p + 1u) : 255u;
        if (e1 == 255u) return lb_token(v, p).nxt;
        ll = 15u + e1;
        pos = p + 2u;
    }
    if (ll > C - pos) return BAD;
    pos += ll;
    if (pos == C) return END;
    if (C - pos < 2u) return BAD;
    pos += 2u;
    if (pos >= C) return BAD;  // a token must follow the match (and a length run needs its byte)
    if ((t & 15u) < 15u) return pos;
    const uint32_t f1 = lb_byte(v, pos);
    if (f1 == 255u) return lb_token(v, p).nxt;
    return pos + 1u >= C ? BAD : pos + 1u;
}

__device__ __forceinline__ LbView lb_view(const uint8_t* src, const LbBlock& B, const uint32_t* nzg, uint32_t cs,
                                          const uint8_t* s) {
    LbView v;
    v.g = src + B.src_off;
    v.s = s;
    v.nzg = nzg;
    v.cs = cs;
    v.C = B.C;
    v.ns = B.C - cs < lb::kStage ? B.C - cs : lb::kStage;
    v.chunk0 = B.chunk0;
    v.nch = B.nchunks;
    return v;
}

}  // namespace

// ---------------------------------------------------------------- classify
__global__ __launch_bounds__(1024) void k_lb_classify(const DecBlock* __restrict__ blk, const DecUnit* __restrict__ units,
                                                      uint32_t nunits, const uint64_t* __restrict__ ucount, LbArgs A) {
    if (ucount) nunits = (uint32_t)min<uint64_t>(*ucount, (uint64_t)nunits);  // a device-built plan's units
    __shared__ uint32_t sh[3][16];
    __shared__ uint32_t carry[3];
    __shared__ uint32_t ntaken;
    const uint32_t t = threadIdx.x;
    if (t < 3) carry[t] = 0;
    if (t == 0) ntaken = 0;
    __syncthreads();
    for (uint32_t base = 0; base < nunits; base += 1024) {
        const uint32_t u = base + t;
        bool cand = false;
        DecBlock B{};
        uint32_t bi = 0;
        if (u < nunits) {
            const DecUnit U = units[u];
            if (U.n == 1) {
                bi = U.first;
                B = blk[bi];
                A.blk_hash[bi] = 0;  // k_lb_run sets it for the blocks it decodes
                cand = !(B.flags & (DB_STORED | DB_LINKED)) && (B.limit >= A.min_limit || B.csize > A.big_csize) &&
                       B.csize > 0 && B.limit <= kLbMaxSteps * kLbStep;
            }
        }
        const uint32_t nch = cand ? (B.csize + kLbChunk - 1) / kLbChunk : 0u;
        uint32_t tot0, tot1;
        const uint32_t p0 = wg_excl_add<uint32_t, 16>(cand ? 1u : 0u, sh[0], tot0) + carry[0];
        const uint32_t p1 = wg_excl_add<uint32_t, 16>(nch, sh[1], tot1) + carry[1];
        // prefixes grow monotonically, so the taken units are a prefix of the candidates
        const bool take = cand && p0 + 1u <= A.lb_cap && p1 + nch <= A.chunk_cap;
        if (u < nunits) A.unit_lb[u] = take ? 1 : 0;
        if (take) {
            LbBlock L;
            L.src_off = B.src_off;
            L.dst_off = B.dst_off;
            L.C = B.csize;
            L.limit = B.limit;
            L.cap = B.cap;
            L.blk = bi;
            L.unit = u;
            L.chunk0 = p1;
            L.nchunks = nch;
            L.pad = 0;
            A.lbt[p0] = L;
            A.lb_err[p0] = 0xFFFFFFFFu;
            atomicMax(&ntaken, p0 + 1u);
            for (uint32_t k = 0; k < nch; ++k) A.chunk_blk[p1 + k] = p0;
        }
        __syncthreads();
        if (t == 0) {
            carry[0] += tot0;
            carry[1] += tot1;
        }
        __syncthreads();
    }
    if (t == 0) {
        const uint32_t n = ntaken;  // the taken candidates are a prefix
        A.ctl->nlb = n;
        A.ctl->nchunks = n ? A.lbt[n - 1].chunk0 + A.lbt[n - 1].nchunks : 0u;
        A.ctl->ntiles = 0;  // k_lbw_plan sets it when the spread execution runs
    }
}

// ---------------------------------------------------------------- granules
__global__ __launch_bounds__(256) void k_lb_gran(const uint8_t* __restrict__ src, LbArgs A) {
    using namespace lb;
    __shared__ uint32_t sm[kGpc];
    const uint32_t c = blockIdx.x;
    if (c >= A.ctl->nchunks) return;
    const LbBlock B = A.lbt[A.chunk_blk[c]];
    const uint8_t* g = src + B.src_off;
    const uint32_t gi = threadIdx.x;
    const uint32_t lo = (c - B.chunk0) * kLbChunk + gi * kGran;
    const uint32_t hi = lo + kGran < B.C ? lo + kGran : B.C;
    uint32_t f = INF;
    for (uint32_t k = lo; k < hi; ++k)
        if (g[k] != 255u) { f = k; break; }
    sm[gi] = f;
    __syncthreads();
    for (uint32_t d = 1; d < kGpc; d <<= 1) {
        const uint32_t o = gi + d < kGpc ? sm[gi + d] : INF;
        __syncthreads();
        sm[gi] = sm[gi] < o ? sm[gi] : o;
        __syncthreads();
    }
    A.nzg[(size_t)c * kGpc + gi] = sm[gi];
}

#if S3HC_LB_TOKV2
// ---------------------------------------------------------------- chunk chains by segment walks
// (round 6; replaces k_lb_exit / k_lb_entry / k_lb_mark's next-token-at-every-position tables and
// their pointer doubling over 8 Ki positions, which cost 1.1 of 2.9 ms at 256 reference frames)
//
// A chunk's kLbWalkT threads each take a segment of segL = ceil(n / kLbWalkT) positions and walk
// the token chain from its first position (speculatively: it may not be a token), marking every
// position visited inside the segment (walk 1); from the first position past the segment each
// walk goes on until it lands on a position some walk 1 marked (it merges with that segment's
// walk from there on) or leaves the chunk (walk 2). The merges link the segments: a chain from any
// position reaches, after the few hops until its first marked position, the chain of that
// position's segment.
//   k_lbt_walk   the walks; per segment (pointer doubling over the segments, 8 levels) the
//                position where its chain leaves the chunk (or END / BAD), and from it the exits
//                of the chunk's first kLbFirstX positions (where a chain enters a chunk unless a
//                literal run spans more than kLbFirstX bytes into it). Marks, exits and both walks'
//                ends go to A.J0 for the next two kernels.
//   k_lbt_entry  per block, over its chunks in order: the true chain's entry into each chunk, one
//                table load per chunk (a walk over the chunk's stored marks otherwise);
//   k_lbt_mark   from its entry: the segments the true chain passes through (reachability by
//                doubling from the entry's first marked position); the true tokens are the reached
//                segments' walk-1 marks from their first true token on, their walk-2 paths and the
//                entry's path to its first mark; then the records, exactly as k_lb_mark wrote them.
// Walks use lb_next (the lz4_flex parse rules, exact for long runs and malformed tokens), so the
// chain's nodes, its malformed last token and every record are the ones the doubling tables gave.
namespace lb {
constexpr uint32_t kWT = kLbWalkT;
constexpr uint32_t kWLv = 8;  // doubling levels: chains over <= kWT segments
static_assert((1u << kWLv) >= kWT, "doubling covers every segment chain");
static_assert(kLbChunk % (32u * kWT) == 0, "whole bitmap words per walking thread");
constexpr uint32_t kWW = kLbChunk / 32u / kWT;  // bitmap words per thread
constexpr uint32_t kBW = kLbChunk / 32u;        // bitmap words per chunk
// per chunk in A.J0 (as u32): marks, then per segment the chain exit, walk 1's end X, walk 2's end M
constexpr uint32_t kGEx = kBW, kGX = kBW + kWT, kGM = kBW + 2u * kWT;
static_assert(2u * (kBW + 3u * kWT) == kLbJ0PerChunk, "A.J0 layout");
}  // namespace lb

namespace {
// Stage block bytes [cs, cs + ns) with aligned 16-byte loads, all of a thread's loads in flight
// before its LDS stores (one HBM round trip); returns s with s[i] = byte cs + i. raw: 16-aligned,
// >= ns + 32 bytes. Loads stay inside the 16-byte granules holding block bytes.
template <uint32_t NT>
__device__ __forceinline__ const uint8_t* lb_stage16(const uint8_t* g, uint32_t cs, uint32_t ns, uint8_t* raw) {
    const uintptr_t a0 = (uintptr_t)(g + cs);
    const uint32_t mis = (uint32_t)(a0 & 15u);
    const uint4* av = (const uint4*)(a0 - mis);
    const uint32_t nv = (mis + ns + 15u) >> 4;
    constexpr uint32_t kL = (lb::kStage + 30u) / 16u / NT + 1u;
    uint4 x[kL];
#pragma unroll
    for (uint32_t k = 0; k < kL; ++k) {
        const uint32_t d = threadIdx.x + k * NT;
        x[k] = d < nv ? av[d] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (uint32_t k = 0; k < kL; ++k) {
        const uint32_t d = threadIdx.x + k * NT;
        if (d < nv) ((uint4*)raw)[d] = x[k];
    }
    return raw + mis;
}
}  // namespace

#ifdef S3HC_LBPROF
#define WK_T(k) { __syncthreads(); const uint64_t n_ = __builtin_amdgcn_s_memtime(); if (threadIdx.x == 0) atomicAdd(&g_lbprof[12 + (k)], (unsigned long long)(n_ - wt_)); wt_ = n_; }
#define WK_MAX(k, h) { atomicMax(&wmx_[k], (h)); }
#define WK_FLUSH() { __syncthreads(); if (threadIdx.x < 4) atomicAdd(&g_lbprof[20 + threadIdx.x], (unsigned long long)wmx_[threadIdx.x]); if (threadIdx.x == 0) atomicAdd(&g_lbprof[24], 1ull); }
#define WK_INIT() __shared__ uint32_t wmx_[4]; if (threadIdx.x < 4) wmx_[threadIdx.x] = 0; uint64_t wt_ = __builtin_amdgcn_s_memtime();
#define WK_CNT(x) ++(x)
#else
#define WK_T(k)
#define WK_MAX(k, h)
#define WK_FLUSH()
#define WK_INIT()
#define WK_CNT(x)
#endif
__global__ __launch_bounds__(lb::kWT) void k_lbt_walk(const uint8_t* __restrict__ src, LbArgs A) {
    using namespace lb;
    WK_INIT()
    __shared__ __attribute__((aligned(16))) uint8_t raw[kStage + 32];
    __shared__ uint32_t bits[kBW];
    __shared__ uint16_t Jg[2][kWT + 1];  // successor segment of a walk (kWT: it left the chunk)
    __shared__ uint32_t ex[2][kWT + 1];  // chain exit, once Jg is terminal
    const uint32_t c = blockIdx.x;
    const uint32_t g = threadIdx.x;
    if (c >= A.ctl->nchunks) return;
    const LbBlock B = A.lbt[A.chunk_blk[c]];
    const uint32_t cs = (c - B.chunk0) * kLbChunk;
    const uint32_t n = B.C - cs < kLbChunk ? B.C - cs : kLbChunk;
    const uint32_t CE = cs + n;
    const LbView v = lb_view(src, B, A.nzg, cs, lb_stage16<kWT>(src + B.src_off, cs, B.C - cs < kStage ? B.C - cs : kStage, raw));
#pragma unroll
    for (uint32_t k = 0; k < kWW; ++k) bits[g + k * kWT] = 0u;
    __syncthreads();
    WK_T(0)
    auto marked = [&](uint32_t P) -> bool {  // P in [cs, CE)
        const uint32_t r = P - cs;
        return ((bits[r >> 5] >> (r & 31u)) & 1u) != 0u;
    };
    // ---- walk 1: the segment's positions on the chain from its first position
    const uint32_t segL = (n + kWT - 1u) / kWT;
    const uint32_t s0 = cs + (g * segL < n ? g * segL : n), s1 = cs + ((g + 1u) * segL < n ? (g + 1u) * segL : n);
    const bool live = s0 < s1;
    uint32_t X = NONE;  // first chain position past the segment, END or BAD
    if (live) {
        // the walk starts kLbWalkLead segments early (unmarked there): by the segment it has mostly
        // fallen in with the token chain, so the walks of earlier segments merge into its marks
        // within a few hops (walk 2's longest path per chunk 21.8 -> see DESIGN 4b)
        uint32_t P = s0 - cs >= kLbWalkLead * segL ? s0 - kLbWalkLead * segL : cs;
        for (;;) {
            if (P >= s0) atomicOr(&bits[(P - cs) >> 5], 1u << ((P - cs) & 31u));
            const uint32_t nx = lb_next(v, P);
            if (nx >= s1) { X = nx; break; }  // (END / BAD compare above every position)
            P = nx;
        }
    }
    __syncthreads();
    WK_T(1)
    // ---- walk 2: until a marked position (merge) or out of the chunk
    uint32_t M = X;
    [[maybe_unused]] uint32_t nh2 = 0;
    if (live)
        while (M < CE) {  // (the mark and the next token are read together)
            const bool mk = marked(M);
            const uint32_t nx = lb_next(v, M);
            if (mk) break;
            M = nx;
            WK_CNT(nh2);
        }
    WK_MAX(0, nh2)
    WK_T(2)
    Jg[0][g] = (uint16_t)(live && M < CE ? (M - cs) / segL : kWT);
    ex[0][g] = live ? (M < CE ? 0u : M) : NONE;
    if (g == 0) {
        Jg[0][kWT] = Jg[1][kWT] = (uint16_t)kWT;
        ex[0][kWT] = ex[1][kWT] = NONE;
    }
    __syncthreads();
    // ---- the chain exit of every segment (pointer doubling: the exit is carried along)
#pragma unroll
    for (uint32_t k = 0; k < kWLv; ++k) {
        const uint32_t j = Jg[k & 1][g];
        uint32_t jn = (uint32_t)kWT, en = ex[k & 1][g];
        if (j != kWT) { jn = Jg[k & 1][j]; en = ex[k & 1][j]; }
        Jg[(k + 1) & 1][g] = (uint16_t)jn;
        ex[(k + 1) & 1][g] = en;
        __syncthreads();
    }
    const uint32_t* exf = ex[kWLv & 1];
    uint32_t* gb = (uint32_t*)(A.J0 + (size_t)c * kLbJ0PerChunk);
#pragma unroll
    for (uint32_t k = 0; k < kWW; ++k) gb[g + k * kWT] = bits[g + k * kWT];
    gb[kGEx + g] = exf[g];
    gb[kGX + g] = X;
    gb[kGM + g] = M;
    WK_T(3)
    if (g < kLbFirstX && g < n) {
        uint32_t P = cs + g;
        [[maybe_unused]] uint32_t nhf = 0;
        while (P < CE) {
            const bool mk = marked(P);
            const uint32_t nx = lb_next(v, P);
            if (mk) break;
            P = nx;
            WK_CNT(nhf);
        }
        WK_MAX(1, nhf)
        A.E[(size_t)c * kLbFirstX + g] = P < CE ? exf[(P - cs) / segL] : P;
    }
    WK_FLUSH()
}

__global__ __launch_bounds__(lb::kWT) void k_lbt_mark(const uint8_t* __restrict__ src, LbArgs A) {
    using namespace lb;
    __shared__ __attribute__((aligned(16))) uint8_t raw[kStage + 32];
    __shared__ uint32_t bits[kBW];
    __shared__ uint16_t Jg[2][kWT + 1];
    __shared__ uint8_t reach[kWT + 1];  // the true chain passes through the segment
    __shared__ uint16_t svfrom[kWT];    // a reached segment's first true token (chunk-relative)
    __shared__ uint16_t tokpos[kTokSlot];
    __shared__ uint32_t shc[4];
    __shared__ uint64_t shs[4];
    __shared__ uint32_t sm0;            // the entry path's first marked position
    __shared__ uint32_t bad_s;
    const uint32_t c = blockIdx.x;
    const uint32_t g = threadIdx.x;
    if (c >= A.ctl->nchunks) return;
    WK_INIT()
    const uint32_t e = A.entry[c];
    if (e == NONE) {  // no token of the block starts in this chunk
        if (g == 0) { A.ntok[c] = 0; A.slsum[c] = 0; A.badrel[c] = NONE; }
        return;
    }
    const LbBlock B = A.lbt[A.chunk_blk[c]];
    const uint32_t cs = (c - B.chunk0) * kLbChunk;
    const uint32_t n = B.C - cs < kLbChunk ? B.C - cs : kLbChunk;
    const uint32_t CE = cs + n;
    // k_lbt_walk's marks and walk ends (loads issued before the staging: both round trips overlap)
    const uint32_t* gb = (const uint32_t*)(A.J0 + (size_t)c * kLbJ0PerChunk);
    uint32_t bw[kWW];
#pragma unroll
    for (uint32_t k = 0; k < kWW; ++k) bw[k] = gb[g + k * kWT];
    const uint32_t X = gb[kGX + g], M = gb[kGM + g];
    const LbView v = lb_view(src, B, A.nzg, cs, lb_stage16<kWT>(src + B.src_off, cs, B.C - cs < kStage ? B.C - cs : kStage, raw));
#pragma unroll
    for (uint32_t k = 0; k < kWW; ++k) bits[g + k * kWT] = bw[k];
    const uint32_t segL = (n + kWT - 1u) / kWT;
    const uint32_t s0 = cs + (g * segL < n ? g * segL : n), s1 = cs + ((g + 1u) * segL < n ? (g + 1u) * segL : n);
    const bool live = s0 < s1;
    Jg[0][g] = (uint16_t)(live && M < CE ? (M - cs) / segL : kWT);
    svfrom[g] = (uint16_t)0xFFFFu;
    reach[g] = 0;
    if (g == 0) {
        Jg[0][kWT] = Jg[1][kWT] = (uint16_t)kWT;
        reach[kWT] = 0;
        bad_s = NONE;
    }
    __syncthreads();
    WK_T(4)
    auto marked = [&](uint32_t P) -> bool {  // P in [cs, CE)
        const uint32_t r = P - cs;
        return ((bits[r >> 5] >> (r & 31u)) & 1u) != 0u;
    };
    auto mark = [&](uint32_t P) {
        const uint32_t r = P - cs;
        atomicOr(&bits[r >> 5], 1u << (r & 31u));
    };
    // ---- the true chain: from the entry to its first marked position m0, then the segment of
    // m0 and every segment reachable from it by merges
    const uint32_t E0 = cs + e;
    if (g == 0) {
        uint32_t P = E0;
        [[maybe_unused]] uint32_t nhe = 0;
        while (P < CE && !marked(P)) { P = lb_next(v, P); WK_CNT(nhe); }
        WK_MAX(2, nhe)
        sm0 = P;
        if (P < CE) {
            const uint32_t h0 = (P - cs) / segL;
            reach[h0] = 1;
            svfrom[h0] = (uint16_t)(P - cs);
        }
    }
    __syncthreads();
    const uint32_t m0 = sm0;
#pragma unroll
    for (uint32_t k = 0; k < kWLv; ++k) {
        const uint32_t h = Jg[k & 1][g];
        if (reach[g]) reach[h] = 1;
        Jg[(k + 1) & 1][g] = Jg[k & 1][h];
        __syncthreads();
    }
    WK_T(5)
    // a reached segment hands its merge point to its successor (that segment's first true token)
    if (reach[g] && live && M < CE) svfrom[(M - cs) / segL] = (uint16_t)(M - cs);
    __syncthreads();
    // marks before a reached segment's first true token are speculative; a segment off the chain
    // is cleared whole
    const uint32_t vf = svfrom[g];
    const bool valid = vf != 0xFFFFu;
    if (live) {
        const uint32_t c1 = valid ? vf : s1 - cs;  // clear [s0, c1) (chunk-relative)
        for (uint32_t q = s0 - cs; q < c1;) {
            const uint32_t w = q >> 5, lo = q & 31u, hi = umin32_lb(32u, c1 - (w << 5));
            const uint32_t mk = (hi == 32u ? ~0u : (1u << hi) - 1u) & (~0u << lo);
            atomicAnd(&bits[w], ~mk);
            q = (w + 1u) << 5;
        }
    }
    __syncthreads();
    // the chain's tokens off the marks: a reached segment's walk-2 path and the entry's path
    [[maybe_unused]] uint32_t nhm = 0;
    if (valid && live)
        for (uint32_t q = X; q < CE && q != M; q = lb_next(v, q)) { mark(q); WK_CNT(nhm); }
    WK_MAX(3, nhm)
    if (g == 0)
        for (uint32_t q = E0; q < CE && q != m0; q = lb_next(v, q)) mark(q);
    __syncthreads();
    WK_T(6)
    // ---- records in stream order (k_lb_mark's layout): thread g lists the marks of its bitmap
    // words at their rank, then parses list entries g, g + kWT, ...
    uint32_t nm = 0;
#pragma unroll
    for (uint32_t k = 0; k < kWW; ++k) nm += (uint32_t)__builtin_popcount(bits[g * kWW + k]);
    uint32_t mtot;
    uint32_t rank = wg_excl_add<uint32_t, kWT / 64>(nm, shc, mtot);
#pragma unroll
    for (uint32_t k = 0; k < kWW; ++k) {
        uint32_t w = bits[g * kWW + k];
        while (w) {
            tokpos[rank++] = (uint16_t)(32u * (g * kWW + k) + (uint32_t)__builtin_ctz(w));
            w &= w - 1u;
        }
    }
    __syncthreads();
    uint32_t cnt = 0;
    uint64_t sl = 0;
    for (uint32_t idx = g; idx < mtot; idx += kWT) {
        const uint32_t r = tokpos[idx];
        const LbTok T = lb_token(v, cs + r);
        if (T.nxt == BAD) {
            bad_s = r;  // the chain's last node (unique)
        } else {
            const uint64_t s1v = (uint64_t)T.ll + T.ml;
            sl += s1v < (uint64_t)B.limit + 1u ? s1v : (uint64_t)B.limit + 1u;
            A.trec[(size_t)c * kTokSlot + idx] =
                make_uint4(T.lit | (T.nxt == END ? 0x80000000u : 0u), T.ll, T.ml, T.off);  // lit < 2^31
            ++cnt;
        }
    }
    uint32_t ctot;
    uint64_t stot;
    (void)wg_excl_add<uint32_t, kWT / 64>(cnt, shc, ctot);
    (void)wg_excl_add<uint64_t, kWT / 64>(sl, shs, stot);
    if (g == 0) {
        A.ntok[c] = ctot;
        A.slsum[c] = stot < 0xFFFFFFFFull ? (uint32_t)stot : 0xFFFFFFFFu;
        A.badrel[c] = bad_s;
    }
    WK_T(7)
    WK_FLUSH()
}
#undef WK_T
#undef WK_MAX
#undef WK_FLUSH
#undef WK_INIT
#undef WK_CNT

// Per block, serial over its chunks: the true chain's entry into each chunk (chunk-relative; NONE
// for chunks a literal run skips), from k_lbt_walk's exit tables.
__global__ void k_lbt_entry(const uint8_t* __restrict__ src, LbArgs A) {
    using namespace lb;
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= A.ctl->nlb) return;
    const LbBlock B = A.lbt[i];
    uint32_t e = 0, c = 0;
    while (c < B.nchunks && e < B.C) {
        const uint32_t cc = e / kLbChunk;
        for (; c < cc; ++c) A.entry[B.chunk0 + c] = NONE;
        const uint32_t cs = cc * kLbChunk, rel = e - cs;
        const size_t ch = (size_t)B.chunk0 + cc;
        A.entry[ch] = rel;
        c = cc + 1u;
        if (rel < kLbFirstX) {
            e = A.E[ch * kLbFirstX + rel];
        } else {
            // a literal run reached past the table: walk over the chunk's marks from HBM
            const uint32_t* gb = (const uint32_t*)(A.J0 + ch * kLbJ0PerChunk);
            const uint32_t n = B.C - cs < kLbChunk ? B.C - cs : kLbChunk, CE = cs + n;
            const uint32_t segL = (n + kWT - 1u) / kWT;
            LbView v;
            v.g = src + B.src_off; v.s = nullptr; v.nzg = A.nzg; v.cs = cs; v.ns = 0; v.C = B.C;
            v.chunk0 = B.chunk0; v.nch = B.nchunks;
            uint32_t P = e;
            while (P < CE) {
                const uint32_t r = P - cs;
                if ((gb[r >> 5] >> (r & 31u)) & 1u) break;
                P = lb_next(v, P);
            }
            e = P < CE ? gb[kGEx + (P - cs) / segL] : P;
        }
    }
    for (; c < B.nchunks; ++c) A.entry[B.chunk0 + c] = NONE;
}
#else  // !S3HC_LB_TOKV2
// ---------------------------------------------------------------- chunk exits
__global__ __launch_bounds__(1024) void k_lb_exit(const uint8_t* __restrict__ src, LbArgs A) {
    using namespace lb;
    __shared__ __attribute__((aligned(16))) uint8_t raw[kStage + 16];
    __shared__ uint32_t nx[kLbChunk];
    __shared__ uint16_t J[kLbChunk];
    const uint32_t c = blockIdx.x;
    if (c >= A.ctl->nchunks) return;
    const LbBlock B = A.lbt[A.chunk_blk[c]];
    const uint32_t cs = (c - B.chunk0) * kLbChunk;
    const uint32_t n = B.C - cs < kLbChunk ? B.C - cs : kLbChunk;
    const uint32_t ce = cs + n;
    const LbView v = lb_view(src, B, A.nzg, cs, lb_stage(src + B.src_off, cs, B.C - cs < kStage ? B.C - cs : kStage, raw));
    __syncthreads();
    for (uint32_t k = 0; k < kPer; ++k) {
        const uint32_t r = threadIdx.x + k * kT;
        if (r < n) {
            const uint32_t nxt = lb_next(v, cs + r);
            nx[r] = nxt;
            const uint16_t j0 = (uint16_t)(nxt < ce ? nxt - cs : r);  // END / BAD / beyond: the chain leaves here
            J[r] = j0;
            A.J0[(size_t)c * kLbChunk + r] = j0;  // k_lb_mark starts from it
        }
    }
    __syncthreads();
    // in-place pointer jumping to the last in-chunk node of each chain (values only move
    // forward along the chain, so reading a fresher value is harmless)
    for (uint32_t lev = 0; lev < 16; ++lev) {
        bool ch = false;
        for (uint32_t k = 0; k < kPer; ++k) {
            const uint32_t r = threadIdx.x + k * kT;
            if (r < n) {
                uint32_t j = J[r];
#pragma unroll
                for (uint32_t h = 0; h < kXHops; ++h) {  // (hops past fresh values between barriers)
                    const uint32_t jj = J[j];
                    if (jj == j) break;
                    j = jj;
                    ch = true;
                }
                J[r] = (uint16_t)j;
            }
        }
        if (!__syncthreads_or(ch)) break;
    }
    for (uint32_t k = 0; k < kPer; ++k) {
        const uint32_t r = threadIdx.x + k * kT;
        if (r < n) A.E[(size_t)c * kLbChunk + r] = nx[J[r]];
    }
}

// ---------------------------------------------------------------- chunk entries
__global__ void k_lb_entry(LbArgs A) {
    using namespace lb;
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= A.ctl->nlb) return;
    const LbBlock B = A.lbt[i];
    uint32_t e = 0, c = 0;
    while (c < B.nchunks && e < B.C) {
        const uint32_t cc = e / kLbChunk;
        for (; c < cc; ++c) A.entry[B.chunk0 + c] = NONE;
        const uint32_t rel = e - cc * kLbChunk;
        A.entry[B.chunk0 + cc] = rel;
        c = cc + 1u;
        e = A.E[(size_t)(B.chunk0 + cc) * kLbChunk + rel];
    }
    for (; c < B.nchunks; ++c) A.entry[B.chunk0 + c] = NONE;
}

// ---------------------------------------------------------------- token marks
// The chain from the chunk's entry is found in three steps instead of pointer doubling over the
// whole chunk: (A) every position learns where its chain leaves its 128-position sub-range (jumping
// inside the sub-range: <= 43 tokens, so a few levels), (B) one thread hops from sub-range to
// sub-range from the entry (<= kSubs hops), (C) one lane per sub-range walks the chain inside it and
// marks the tokens (about 20 hops). Positions are chunk-relative; J0[r] == r: the chain leaves
// the chunk (or ends) after r.
namespace lb {
constexpr uint32_t kSub = 128;                  // positions per sub-range
constexpr uint32_t kSubs = kLbChunk / kSub;     // sub-ranges per chunk
static_assert(kSubs <= 64, "one lane per sub-range");
}  // namespace lb
__global__ __launch_bounds__(1024) void k_lb_mark(const uint8_t* __restrict__ src, LbArgs A) {
    using namespace lb;
    __shared__ __attribute__((aligned(16))) uint8_t raw[kStage + 16];
    __shared__ uint16_t J[kLbChunk], X[kLbChunk];
    __shared__ uint8_t mk[kLbChunk];
    __shared__ uint16_t first[kSubs];
    __shared__ uint16_t tokpos[kTokSlot];  // marked positions in order
    __shared__ uint32_t shc[16];
    __shared__ uint64_t shs[16];
    __shared__ uint32_t bad_s;
    const uint32_t c = blockIdx.x;
    const bool live = c < A.ctl->nchunks;
    const uint32_t e = live ? A.entry[c] : NONE;
    if (e == NONE) {  // no token of the block starts in this chunk (or a chunk beyond the count)
        if (threadIdx.x == 0) { A.ntok[c] = 0; A.slsum[c] = 0; A.badrel[c] = NONE; }
        return;
    }
#ifdef S3HC_LBPROF
    uint64_t mt = __builtin_amdgcn_s_memtime();
#define MK_T(k) { __syncthreads(); const uint64_t n_ = __builtin_amdgcn_s_memtime(); if (threadIdx.x == 0) atomicAdd(&g_lbprof[12 + (k)], (unsigned long long)(n_ - mt)); mt = n_; }
#else
#define MK_T(k)
#endif
    const LbBlock B = A.lbt[A.chunk_blk[c]];
    const uint32_t cs = (c - B.chunk0) * kLbChunk;
    const uint32_t n = B.C - cs < kLbChunk ? B.C - cs : kLbChunk;
    // the chain table's loads are issued before the input staging so both HBM round trips overlap
    uint16_t j0r[kPer];
#pragma unroll
    for (uint32_t k = 0; k < kPer; ++k) {
        const uint32_t r = threadIdx.x + k * kT;
        j0r[k] = r < n ? A.J0[(size_t)c * kLbChunk + r] : (uint16_t)0;
    }
    const LbView v = lb_view(src, B, A.nzg, cs, lb_stage(src + B.src_off, cs, B.C - cs < kStage ? B.C - cs : kStage, raw));
    if (threadIdx.x == 0) bad_s = NONE;
    if (threadIdx.x < kSubs) first[threadIdx.x] = 0xFFFFu;
#pragma unroll
    for (uint32_t k = 0; k < kPer; ++k) {
        const uint32_t r = threadIdx.x + k * kT;
        if (r < n) {
            J[r] = j0r[k];
            X[r] = j0r[k];
            mk[r] = 0;
        }
    }
    __syncthreads();
    MK_T(0)
    // (A) X[r]: the first chain node after r outside r's sub-range, or the node the chain ends on
    // inside it (values only move forward along the chain: reading a fresher one is harmless)
    for (uint32_t lev = 0; lev < 8; ++lev) {
        bool ch = false;
        for (uint32_t k = 0; k < kPer; ++k) {
            const uint32_t r = threadIdx.x + k * kT;
            if (r < n) {
                uint32_t j = X[r];
                bool mv = false;
#pragma unroll
                for (uint32_t h = 0; h < kXHops; ++h) {
                    if (j == r || j / kSub != r / kSub) break;
                    const uint32_t jj = X[j];
                    if (jj == j) break;
                    j = jj;
                    mv = true;
                }
                if (mv) { X[r] = (uint16_t)j; ch = true; }
            }
        }
        if (!__syncthreads_or(ch)) break;
    }
    MK_T(1)
    // (B) the chain's first node in each sub-range it visits
    if (threadIdx.x == 0) {
        uint32_t cur = e;
        while (true) {
            first[cur / kSub] = (uint16_t)cur;
            const uint32_t nx = X[cur];
            if (nx == cur || nx / kSub == cur / kSub) break;  // the chain ends inside this sub-range
            cur = nx;
        }
    }
    __syncthreads();
    // (C) lane s walks the chain inside sub-range s
    if (threadIdx.x < kSubs && first[threadIdx.x] != 0xFFFFu) {
        uint32_t cur = first[threadIdx.x];
        while (true) {
            mk[cur] = 1;
            const uint32_t nx = J[cur];
            if (nx == cur || nx / kSub != threadIdx.x) break;
            cur = nx;
        }
    }
    __syncthreads();
    MK_T(2)
    // the chunk's tokens in position order: the marked positions are listed at their rank (from
    // the marks alone: the one marked position that is not a token — the malformed token ending a
    // corrupt chain — is the chain's last node, after every token), then thread t parses list
    // entries t, t + kT, ... and writes their records at that rank in the chunk's slot of trec,
    // so k_lb_seq only scans
    const uint32_t r0 = kPer * threadIdx.x;
    uint32_t nm = 0;
#pragma unroll
    for (uint32_t k = 0; k < kPer; ++k) nm += (r0 + k < n && mk[r0 + k]) ? 1u : 0u;
    uint32_t mtot;
    uint32_t rank = wg_excl_add<uint32_t, 16>(nm, shc, mtot);
#pragma unroll
    for (uint32_t k = 0; k < kPer; ++k)
        if (r0 + k < n && mk[r0 + k]) tokpos[rank++] = (uint16_t)(r0 + k);
    __syncthreads();
    uint32_t cnt = 0;
    uint64_t sl = 0;
    for (uint32_t idx = threadIdx.x; idx < mtot; idx += kT) {
        const uint32_t r = tokpos[idx];
        const LbTok T = lb_token(v, cs + r);
        if (T.nxt == BAD) {
            bad_s = r;  // the chain's last node (unique)
        } else {
            const uint64_t s1 = (uint64_t)T.ll + T.ml;
            sl += s1 < (uint64_t)B.limit + 1u ? s1 : (uint64_t)B.limit + 1u;
            A.trec[(size_t)c * kTokSlot + idx] =
                make_uint4(T.lit | (T.nxt == END ? 0x80000000u : 0u), T.ll, T.ml, T.off);  // lit < 2^31
            ++cnt;
        }
    }
    MK_T(3)
    uint32_t ctot;
    uint64_t stot;
    (void)wg_excl_add<uint32_t, 16>(cnt, shc, ctot);
    (void)wg_excl_add<uint64_t, 16>(sl, shs, stot);
    MK_T(4)
#undef MK_T
    if (threadIdx.x == 0) {
        A.ntok[c] = ctot;
        A.slsum[c] = stot < 0xFFFFFFFFull ? (uint32_t)stot : 0xFFFFFFFFu;
        A.badrel[c] = bad_s;
    }
}
#endif  // S3HC_LB_TOKV2

// ---------------------------------------------------------------- sequence table
__device__ __forceinline__ uint32_t lb_check(uint64_t produced, uint32_t ll, uint32_t ml, uint32_t off, bool last,
                                             uint32_t limit, uint32_t cap) {
    // dec_block's check(): precedence lowest first, later conditions override
    const int64_t have = (int64_t)produced + ll;
    uint32_t st = S3HC_OK;
    st = (!last && (int64_t)ml > (int64_t)cap - have) ? S3HC_DST_TOO_SMALL : st;
    st = (!last && (int64_t)ml > (int64_t)limit - have) ? S3HC_CORRUPT : st;
    st = (!last && (off == 0 || (int64_t)off > have)) ? S3HC_CORRUPT : st;
    st = ((int64_t)ll > (int64_t)cap - (int64_t)produced) ? S3HC_DST_TOO_SMALL : st;
    st = ((int64_t)ll > (int64_t)limit - (int64_t)produced) ? S3HC_CORRUPT : st;
    return st;
}

// 256 threads per chunk: the records are read and the table written rank-strided (rank t + 256 k:
// coalesced), the output offsets scanned over contiguous ranks through LDS (round 6: the
// 1024-thread form read and wrote three consecutive records per thread)
namespace lb {
constexpr uint32_t kSeqT = 256;
constexpr uint32_t kSeqK = (kTokSlot + kSeqT - 1u) / kSeqT;
}
__global__ __launch_bounds__(lb::kSeqT) void k_lb_seq(const uint8_t* __restrict__ src, LbArgs A) {
    using namespace lb;
    __shared__ uint64_t shs[kSeqT / 64];
    __shared__ uint64_t opos[kSeqK * kSeqT];  // per rank: clamped output bytes, then output offset
    const uint32_t c = blockIdx.x;
    if (c >= A.ctl->nchunks || A.entry[c] == NONE) return;
    const uint32_t bi = A.chunk_blk[c];
    const LbBlock B = A.lbt[bi];
    const uint32_t cs = (c - B.chunk0) * kLbChunk;
    const uint32_t ntc = A.ntok[c];
    const uint32_t t = threadIdx.x;
    const uint4* tr = A.trec + (size_t)c * kTokSlot;
    auto clampsl = [&](uint32_t ll, uint32_t ml) -> uint64_t {
        const uint64_t s1 = (uint64_t)ll + ml;
        return s1 < (uint64_t)B.limit + 1u ? s1 : (uint64_t)B.limit + 1u;
    };
    uint4 rv[kSeqK];
#pragma unroll
    for (uint32_t k = 0; k < kSeqK; ++k) {
        const uint32_t i = t + kSeqT * k;
        rv[k] = i < ntc ? tr[i] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (uint32_t k = 0; k < kSeqK; ++k) {
        const uint32_t i = t + kSeqT * k;
        if (i < ntc) opos[i] = clampsl(rv[k].y, rv[k].z);
    }
    __syncthreads();
    const uint32_t K = (ntc + kSeqT - 1u) / kSeqT;
    const uint32_t i0 = umin32_lb(ntc, K * t), i1 = umin32_lb(ntc, i0 + K);
    uint64_t sl = 0;
    for (uint32_t i = i0; i < i1; ++i) sl += opos[i];
    uint64_t stot;
    const uint64_t opre = wg_excl_add<uint64_t, kSeqT / 64>(sl, shs, stot);
    const uint64_t tb0 = A.tokbase[B.chunk0];
    const uint64_t ob0 = A.outbase[B.chunk0];
    const uint64_t gbase = A.tokbase[c];
    const uint32_t brank0 = (uint32_t)(gbase - tb0);
    {
        uint64_t produced = A.outbase[c] - ob0 + opre;
        for (uint32_t i = i0; i < i1; ++i) {
            const uint64_t v = opos[i];
            opos[i] = produced;
            produced += v;
        }
    }
    __syncthreads();
    uint32_t bad = 0xFFFFFFFFu;
#pragma unroll
    for (uint32_t k = 0; k < kSeqK; ++k) {
        const uint32_t rank = t + kSeqT * k;
        if (rank >= ntc) continue;
        const uint64_t produced = opos[rank];
        const uint4 rec = rv[k];
        LbTok S;
        S.lit = rec.x & 0x7FFFFFFFu; S.ll = rec.y; S.ml = rec.z; S.off = rec.w;
        const bool last = (rec.x >> 31) != 0;
        const uint32_t st = lb_check(produced, S.ll, S.ml, S.off, last, B.limit, B.cap);
        const uint32_t br = brank0 + rank;
        if (st != S3HC_OK && bad == 0xFFFFFFFFu) bad = (br << 3) | st;
        A.seq4[gbase + rank] = make_uint4(produced < 0xFFFFFFFFull ? (uint32_t)produced : 0xFFFFFFFFu, S.lit,
                                          S.ll, S.ml);
        A.seqoff[gbase + rank] = (uint16_t)S.off;
        // execution steps whose first byte this sequence produces
        const uint64_t sl1 = (uint64_t)S.ll + S.ml;
        if (st == S3HC_OK && sl1) {
            const uint64_t r_lo = (produced + kLbStep - 1) / kLbStep, r_hi = (produced + sl1 - 1) / kLbStep;
            for (uint64_t q = r_lo; q <= r_hi && q < kLbMaxSteps; ++q) A.rfirst[(size_t)bi * kLbMaxSteps + q] = br;
        }
    }
    if (bad != 0xFFFFFFFFu) atomicMin(&A.lb_err[bi], bad);
    if (threadIdx.x == 0) {
        const uint32_t br = A.badrel[c];
        if (br != NONE) {
            // the malformed token ending the chain: after every sequence of the block
            LbView v;  // one token, read from HBM
            v.g = src + B.src_off; v.s = nullptr; v.nzg = A.nzg; v.cs = cs; v.ns = 0; v.C = B.C;
            v.chunk0 = B.chunk0; v.nch = B.nchunks;
            const LbTok S = lb_token(v, cs + br);
            const uint64_t pr = A.outbase[c] - ob0 + stot;
            uint32_t st = S3HC_CORRUPT, rk = brank0 + ntc;
            if (S.late == 1) {  // literal checks, then the cut-off offset / length run
                st = ((int64_t)S.ll > (int64_t)B.cap - (int64_t)pr) ? S3HC_DST_TOO_SMALL : st;
                st = ((int64_t)S.ll > (int64_t)B.limit - (int64_t)pr) ? S3HC_CORRUPT : st;
            } else if (S.late == 2) {  // a full sequence, then the missing token
                const uint32_t sc = lb_check(pr, S.ll, S.ml, S.off, false, B.limit, B.cap);
                st = sc != S3HC_OK ? sc : S3HC_CORRUPT;
                rk += sc != S3HC_OK ? 0u : 1u;
            }
            atomicMin(&A.lb_err[bi], (rk << 3) | st);
        }
    }
}

// ---------------------------------------------------------------- finish parse
// size and status of LB block i (< nlb); returns the status, *size_out the decoded bytes (0 unless OK)
__device__ __forceinline__ uint32_t lb_fin_block(const LbArgs& A, uint32_t i, uint32_t* __restrict__ blk_out,
                                                 int32_t* __restrict__ blk_status, uint32_t* size_out) {
    const LbBlock B = A.lbt[i];
    const uint32_t cl = B.chunk0 + B.nchunks - 1;
    const uint64_t size = A.outbase[cl] + A.slsum[cl] - A.outbase[B.chunk0];
    const uint32_t err = A.lb_err[i];
    const uint32_t stat = err == 0xFFFFFFFFu ? (uint32_t)S3HC_OK : (err & 7u);
    A.lb_size[i] = stat == S3HC_OK ? (uint32_t)size : 0u;
    A.lb_stat[i] = stat;
    A.lb_tok0[i] = (uint32_t)A.tokbase[B.chunk0];
    A.lb_ntok[i] = (uint32_t)(A.tokbase[cl] + A.ntok[cl] - A.tokbase[B.chunk0]);
    blk_out[B.blk] = stat == S3HC_OK ? (uint32_t)size : 0u;
    blk_status[B.blk] = (int32_t)stat;
    *size_out = stat == S3HC_OK ? (uint32_t)size : 0u;
    return stat;
}
__global__ void k_lb_fin(LbArgs A, uint32_t* __restrict__ blk_out, int32_t* __restrict__ blk_status) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t size;
    if (i < A.ctl->nlb) (void)lb_fin_block(A, i, blk_out, blk_status, &size);
}

// ---------------------------------------------------------------- execute
// One 1024-thread workgroup per block writes the block in kLbStep-byte steps, in order: 15
// waves decode, the 16th hashes. LDS keeps a 64 KiB ring of the block's recent output (match
// sources) and the step's sequences. Each byte of a step gets its value right away when it is a
// literal or its match source lies before the step (the ring still holds [R - 64 KiB, R) until
// the step stores its own bytes, and LZ4 offsets are < 64 KiB); otherwise it gets a pointer to
// its source inside the step, and the pointers are jumped (a final source gives the value) until
// every byte is final: every chain ends in a literal or a byte before the step, so no byte is
// left over. Then the step is flushed.
//
// The hashing wave runs xxh32 (seed 0) over the block's output behind the decode: in each
// barrier phase of a step it hashes a slice of the bytes finished by earlier steps (from the
// LDS ring), sized to that phase's length, so its serial chain hides in the other waves' LDS
// and memory phases; the tail and the final avalanche follow the last flush. The result goes to blk_hash[blk] (1 << 32 | hash): when the
// block is its frame's only block this is the frame's content checksum, and k_dframe_close
// skips its own serial pass over the frame (0.7 ms per MiB).
namespace {
constexpr uint32_t XH1 = 2654435761U, XH2 = 2246822519U, XH3 = 3266489917U, XH4 = 668265263U, XH5 = 374761393U;
__device__ __forceinline__ uint32_t xh_rotl(uint32_t x, int r) { return __builtin_amdgcn_alignbit(x, x, 32 - r); }
__device__ __forceinline__ uint32_t xh_round(uint32_t acc, uint32_t in) { return xh_rotl(acc + in * XH2, 13) * XH1; }
typedef uint32_t u32_unaligned __attribute__((aligned(1)));
}  // namespace

__global__ __launch_bounds__(1024) void k_lb_run(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, LbArgs A) {
    using namespace lb;
    __shared__ __attribute__((aligned(16))) uint8_t ring[kRing];
    __shared__ __attribute__((aligned(16))) uint32_t ptr[kLbStep];
    __shared__ __attribute__((aligned(16))) uint16_t marks[kLbStep];
    __shared__ __attribute__((aligned(16))) uint4 sq[kMaxSeqS];
    __shared__ uint16_t so[kMaxSeqS];
    __shared__ uint32_t rf[kLbMaxSteps + 1];
    __shared__ __attribute__((aligned(16))) uint32_t shm[16];
    __shared__ uint32_t jflag[3];
    __shared__ uint32_t xb_ctr;    // S3HC_LB_XBAR: arrivals at the decoding waves' barriers
    __shared__ uint32_t x_final;   // bytes of the block final in the ring (whole steps), for the hashing wave
    __shared__ uint32_t x_hashed;  // stripes the hashing wave has hashed (ring slots it no longer reads)
    const uint32_t i = blockIdx.x;
    if (i >= A.ctl->nlb || A.lb_stat[i] != S3HC_OK) return;
    if (A.wcap && A.wbase[i] != lb::NONE) return;  // spread execution decodes it (k_lbw_*)
    const LbBlock B = A.lbt[i];
    const uint32_t size = A.lb_size[i];
    const uint32_t tok0 = A.lb_tok0[i], ntok = A.lb_ntok[i];
    const uint8_t* g = src + B.src_off;
    uint8_t* ob = dst + B.dst_off;
    const uint32_t t = threadIdx.x;
    const bool dec = t < kXT;  // decoding thread (else: the hashing wave)
    const int lane = lane64();
    constexpr uint32_t kMask = kRing - 1;
    const uint32_t nsteps = (size + kLbStep - 1) / kLbStep;
#ifdef S3HC_LBPROF
    uint64_t lbp[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t lbt = __builtin_amdgcn_s_memtime();
    // phase k accumulates the time since the previous mark (0: step loop overhead)
#define LB_T(k) { const uint64_t n_ = __builtin_amdgcn_s_memtime(); lbp[(k) == 0 ? 9 : (k) - 1] += n_ - lbt; lbt = n_; }
#define LB_ADD(k, v) lbp[k] += (v)
#else
#define LB_T(k)
#define LB_ADD(k, v)
#endif
    // hashing wave state: lane a = lane & 3 runs accumulator a (every lane computes; lanes of a
    // quad share addresses), hs = stripes hashed so far
    const uint32_t ha = (uint32_t)lane & 3u;
    uint32_t hacc = ha == 0 ? XH1 + XH2 : (ha == 1 ? XH2 : (ha == 2 ? 0u : 0u - XH1));
    uint32_t hs = 0;
    const uint32_t hns = size >> 4;
    // hash stripes [hs, min(avail / 16, hs + budget)) of the finished output, read from the LDS
    // ring (aligned dwords: ring slots are output positions mod 64 KiB; the hashing wave lags the
    // decode by about one step, far less than the ring's 8)
#if defined(S3HC_LB_NOHASH) || S3HC_LB_XBAR  // (S3HC_LB_NOHASH diagnostic builds: k_dframe_close hashes;
#define LB_HASH(avail, budget)                   // S3HC_LB_XBAR: the hashing wave runs its own loop)
#else
#define LB_HASH(avail, budget)                                                                  \
    if (!dec) {                                                                                 \
        uint32_t lim_ = (avail) >> 4;                                                           \
        lim_ = lim_ < hns ? lim_ : hns;                                                         \
        lim_ = lim_ < hs + (budget) ? lim_ : hs + (budget);                                     \
        for (; hs + 16u <= lim_; hs += 16u) {                                                   \
            /* lane 4k + a loads stripe k's dword a and multiplies it by P2 (off the chain, one */ \
            /* load and one multiply for 16 stripes); the chain then only adds, rotates and     */ \
            /* multiplies by P1                                                                 */ \
            const uint32_t mv_ = *(const uint32_t*)(ring + ((16u * hs + 4u * (uint32_t)lane) & kMask)) * XH2; \
            uint32_t m_[16];                                                                    \
            _Pragma("unroll") for (uint32_t k = 0; k < 16; ++k) m_[k] = __shfl(mv_, (int)(4u * k + ha)); \
            _Pragma("unroll") for (uint32_t k = 0; k < 16; ++k) hacc = xh_rotl(hacc + m_[k], 13) * XH1; \
        }                                                                                       \
        for (; hs < lim_; ++hs) hacc = xh_round(hacc, *(const uint32_t*)(ring + ((16u * hs + 4u * ha) & kMask))); \
    }
#endif
    // step q covers sequences [rf[q], rf[q+1]) (+1 when the next step starts inside one)
    for (uint32_t q = t; q <= nsteps; q += kXWG)
        rf[q] = q < nsteps ? A.rfirst[(size_t)i * kLbMaxSteps + q] : ntok;
    if (t == 0) {
        xb_ctr = 0;
        x_final = 0;
        x_hashed = 0;
    }
    __syncthreads();
    // sequences of a step: loaded into registers one step ahead, stored (with the start marks)
    // into LDS once the current step no longer needs them (kMaxSeqS <= 3 x kXT)
    static_assert(kMaxSeqS <= 3 * kXT, "three sequences per thread and step");
    uint4 pe0 = make_uint4(0, 0, 0, 0), pe1 = pe0, pe2 = pe0;
    uint32_t po0 = 0, po1 = 0, po2 = 0;
#define LB_STEP_SEQS(q, s0, ns)                                              \
    const uint32_t s0 = rf[q];                                               \
    const uint32_t ns = ((q) + 1 < nsteps ? rf[(q) + 1] + 1u : ntok) - s0 < kMaxSeqS \
                            ? ((q) + 1 < nsteps ? rf[(q) + 1] + 1u : ntok) - s0      \
                            : kMaxSeqS;
#define LB_PREFETCH(q)                                                                   \
    if (dec) {                                                                           \
        LB_STEP_SEQS(q, s0p, nsp)                                                        \
        const uint32_t j0 = t, j1 = t + kXT, j2 = t + 2 * kXT;                           \
        const uint32_t g0 = tok0 + s0p + (j0 < nsp ? j0 : 0u), g1 = tok0 + s0p + (j1 < nsp ? j1 : 0u); \
        const uint32_t g2 = tok0 + s0p + (j2 < nsp ? j2 : 0u);                           \
        pe0 = A.seq4[g0]; pe1 = A.seq4[g1]; pe2 = A.seq4[g2];                            \
        po0 = A.seqoff[g0]; po1 = A.seqoff[g1]; po2 = A.seqoff[g2];                      \
    }
#define LB_PUT(j, pe, po, R)                                                             \
    if ((j) < nsi) {                                                                     \
        sq[j] = pe;                                                                      \
        so[j] = (uint16_t)(po);                                                          \
        const uint32_t rel_ = (pe).x > (R) ? (pe).x - (R) : 0u;                          \
        if (rel_ < kLbStep && ((j) == 0 || (pe).x > (R))) marks[rel_] = (uint16_t)((j) + 1); \
    }
#define LB_INSTALL(q)                                                                    \
    if (dec) {                                                                           \
        LB_STEP_SEQS(q, s0i, nsi)                                                        \
        const uint32_t Rq = (q) * kLbStep;                                               \
        (void)s0i;                                                                       \
        LB_PUT(t, pe0, po0, Rq) LB_PUT(t + kXT, pe1, po1, Rq) LB_PUT(t + 2 * kXT, pe2, po2, Rq) \
    }
    if (dec) ((uint4*)marks)[t] = make_uint4(0, 0, 0, 0);  // kLbStep u16 = kXT x 16 B
    LB_PREFETCH(0)
    __syncthreads();
    LB_INSTALL(0)
    if (1 < nsteps) LB_PREFETCH(1)
    __syncthreads();
#if S3HC_LB_XBAR
    // From here the decoding waves synchronise among themselves (lb_xbar) and the hashing wave
    // runs free: it hashes every whole step the decoders publish (x_final), from the ring, and
    // publishes its progress (x_hashed); the decoders wait for it only before overwriting ring
    // slots it has not read (it trails by about a step; the ring holds eight). In rounds 2-5 it
    // took part in every barrier of the step loop with slices sized to the phases, and the phases
    // it overran cost 0.28 of k_lb_run's 1.6 ms at 256 reference frames.
    uint32_t xtgt = 0;
    constexpr uint32_t kXW = kXT / 64u;
#define LB_SYNC() lb_xbar(&xb_ctr, xtgt, kXW)
    if (!dec) {
#ifndef S3HC_LB_NOHASH
        for (uint32_t n = 0; hs < hns && n < (1u << 26);) {
            uint32_t lim = __hip_atomic_load(&x_final, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) >> 4;
            lim = lim < hns ? lim : hns;
            if (lim <= hs) {
                __builtin_amdgcn_s_sleep(1);
                ++n;
                continue;
            }
            for (; hs + 16u <= lim; hs += 16u) {
                // lane 4k + a loads stripe k's dword a and multiplies it by P2 (off the chain)
                const uint32_t mv = *(const uint32_t*)(ring + ((16u * hs + 4u * (uint32_t)lane) & kMask)) * XH2;
                uint32_t m[16];
#pragma unroll
                for (uint32_t k = 0; k < 16; ++k) m[k] = __shfl(mv, (int)(4u * k + ha));
#pragma unroll
                for (uint32_t k = 0; k < 16; ++k) hacc = xh_rotl(hacc + m[k], 13) * XH1;
            }
            for (; hs < lim; ++hs) hacc = xh_round(hacc, *(const uint32_t*)(ring + ((16u * hs + 4u * ha) & kMask)));
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            if (lane == 0) __hip_atomic_store(&x_hashed, hs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        // every step is final: the tail (from the ring) and the avalanche
        for (uint32_t n = 0; n < (1u << 26) && __hip_atomic_load(&x_final, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < size; ++n)
            __builtin_amdgcn_s_sleep(1);
        const int qb = lane & ~3;
        const uint32_t v1 = __shfl(hacc, qb), v2 = __shfl(hacc, qb + 1), v3 = __shfl(hacc, qb + 2),
                       v4 = __shfl(hacc, qb + 3);
        if (lane == 0) {
            uint32_t h = size >= 16 ? xh_rotl(v1, 1) + xh_rotl(v2, 7) + xh_rotl(v3, 12) + xh_rotl(v4, 18) : XH5;
            h += size;
            uint32_t p = hns * 16u;
            auto rb = [&](uint32_t x) -> uint32_t { return ring[x & kMask]; };
            for (; p + 4u <= size; p += 4u)
                h = xh_rotl(h + (rb(p) | rb(p + 1) << 8 | rb(p + 2) << 16 | rb(p + 3) << 24) * XH3, 17) * XH4;
            for (; p < size; ++p) h = xh_rotl(h + rb(p) * XH5, 11) * XH1;
            h ^= h >> 15;
            h *= XH2;
            h ^= h >> 13;
            h *= XH3;
            h ^= h >> 16;
            A.blk_hash[B.blk] = (1ull << 32) | h;
        }
#endif
        return;
    }
#else
#define LB_SYNC() __syncthreads()
#endif
#if S3HC_LB_OWNFUSE
    uint32_t os = 0, oinc = 0;  // the next step's owner scan: halves done; this lane's wave maximum
    uint4 om4 = make_uint4(0, 0, 0, 0);
    bool own_sync = false;
#endif
    for (uint32_t q = 0; q < nsteps; ++q) {
        const uint32_t R = q * kLbStep;
        LB_T(0);
        LB_ADD(7, 1);
        // owner of each byte: running max of the start marks (thread t: bytes 8t .. 8t+7)
        // (owners written over the marks, then read with the interleaved byte mapping; the
        // hashing wave's marks are zero)
#if S3HC_LB_OWNFUSE
        // (steps after the first: the previous step's jumping rounds ran the scan, os == 2;
        // own_sync: its owners were stored after the rounds' last barrier)
        if (q == 0) {
            const uint4 own = lb_owners_b(dec ? ((const uint4*)marks)[t] : make_uint4(0, 0, 0, 0), shm, [&] { LB_SYNC(); });
            if (dec) ((uint4*)marks)[t] = own;
            LB_SYNC();
        } else if (own_sync) {
            LB_SYNC();
        }
        os = 0;
        own_sync = false;
#else
        const uint4 own = lb_owners_b(dec ? ((const uint4*)marks)[t] : make_uint4(0, 0, 0, 0), shm, [&] { LB_SYNC(); });
        if (dec) ((uint4*)marks)[t] = own;
        LB_SYNC();
#endif
        // (a hashing wave more than 3 steps behind catches up here: the ring keeps 8)
        LB_HASH(R, R - 16u * hs > 3u * kLbStep ? (R - 16u * hs - 2u * kLbStep) / 16u
                                                : (R - 16u * hs > kHashLag ? kHashClassify : 0u))
        // classify the bytes (thread t: bytes t + kXT*j, so lanes touch consecutive bytes):
        // literal (input address), source before the step (ring value: the ring still holds
        // [R - 64 KiB, R) until this step's bytes are stored below, and LZ4 offsets are
        // < 64 KiB), source inside the step (pointer). An overlapping copy's source is taken in
        // its first period, or in its latest period before the step when there is one.
        LB_T(1);
        uint32_t la[kXPer], pv[kXPer], vb[kXPer];
        uint32_t litm = 0;
#pragma unroll
        for (uint32_t j = 0; j < kXPer; ++j) {
            const uint32_t l = t + kXT * j;
            const uint32_t x = R + l;
            pv[j] = FIN;
            la[j] = 0;
            vb[j] = 0;
            if (dec && x < size) {
                const uint32_t k = marks[l] - 1u;
                const uint4 e = sq[k];
                const uint32_t rel = x - e.x;
                if (rel < e.z) {
                    la[j] = e.y + rel;
                    litm |= 1u << j;
                } else {
                    const uint32_t off = so[k];
                    uint32_t y = x - off;
                    const uint32_t ee = rel - e.z;  // position inside the match
                    if (y >= R && ee >= off) {
                        const uint32_t m0 = e.x + e.z;
                        const uint32_t yf = m0 - off + ee % off;
                        y = yf < R ? x - ((x - R) / off + 1u) * off : yf;
                    }
                    if (y >= R) pv[j] = y - R;
                    else vb[j] = ring[y & kMask];
                }
            }
        }
        // literal loads (coalesced across lanes), all issued before the first use
        uint32_t lv[kXPer];
#pragma unroll
        for (uint32_t j = 0; j < kXPer; ++j) lv[j] = g[(litm >> j) & 1u ? la[j] : 0u];
#pragma unroll
        for (uint32_t j = 0; j < kXPer; ++j) vb[j] = (litm >> j) & 1u ? lv[j] & 0xFFu : vb[j];
        LB_T(2);
#if S3HC_LB_XBAR
        // the ring slots this step overwrites ([R + kLbStep - kRing, R)'s) were hashed
        if (t == 0 && R + kLbStep > kRing)
            for (uint32_t n = 0; n < (1u << 26) &&
                                 16u * __hip_atomic_load(&x_hashed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) + kRing < R + kLbStep;
                 ++n)
                __builtin_amdgcn_s_sleep(1);
#endif
        LB_SYNC();  // every read of the ring slots this step overwrites, and of marks/sq, is done
        if (dec) {
#pragma unroll
            for (uint32_t j = 0; j < kXPer; ++j) {
                const uint32_t l = t + kXT * j;
                ring[(R + l) & kMask] = (uint8_t)vb[j];
                ptr[l] = pv[j] == FIN ? (VALF | vb[j]) : pv[j];  // a final byte's entry carries its value
            }
            ((uint4*)marks)[t] = make_uint4(0, 0, 0, 0);
        }
        if (t == 0) jflag[0] = 0u;
        LB_HASH(R, kHashStores)
        LB_SYNC();
        LB_T(3);
        if (q + 1 < nsteps) LB_INSTALL(q + 1)
        if (q + 2 < nsteps) LB_PREFETCH(q + 2)
        LB_HASH(R, kHashInstall)
        LB_T(4);
        // chains inside the step: each round every pending byte reads its source's pointer; a
        // final source gives the value, a pending one is jumped over (pointer doubling). A
        // thread's pointers stay in registers (it is their only writer); values are stored
        // before the pointers that mark them final (a wave's LDS operations complete in order).
        uint32_t pend = 0;
#pragma unroll
        for (uint32_t j = 0; j < kXPer; ++j) pend |= (pv[j] != FIN ? 1u : 0u) << j;
        // one barrier per round: threads still pending after the round raise jflag[it % 3];
        // thread 0 clears the next round's flag before the barrier (nobody reads or raises it
        // until after the barrier), jflag[0] was cleared before the stores barrier
        for (uint32_t it = 0; it < 20; ++it) {
#ifdef S3HC_LBPROF
            const uint64_t tb1 = __builtin_amdgcn_s_memtime();
#endif
#if S3HC_LB_OWNFUSE
            // the next step's owner scan, one half per round: its marks were installed before
            // round 0's barrier, the wave maxima are read after a later one, and the owners'
            // stores precede this round's barrier
            if (q + 1 < nsteps && it >= 1 && os < 2) {
                if (os == 0) {
                    om4 = ((const uint4*)marks)[t];
                    oinc = lb_own1(om4, shm);
                } else {
                    ((uint4*)marks)[t] = lb_own2(om4, oinc, shm);
                }
                ++os;
            }
#endif
            // up to kJumpHops hops per round between barriers: pointers other threads stored in
            // this round are read as soon as they land (LDS), which only shortens the chains
            // (a final entry is VALF | byte value: one gather gives both the state and the value)
            for (uint32_t h = 0; h < kJumpHops && pend; ++h) {
                uint32_t pp[kXPer];
#pragma unroll
                for (uint32_t j = 0; j < kXPer; ++j) pp[j] = (pend >> j) & 1u ? ptr[pv[j]] : 0u;
                uint32_t fin = 0;
#pragma unroll
                for (uint32_t j = 0; j < kXPer; ++j) {
                    if ((pend >> j) & 1u) {
                        const bool f = (pp[j] & VALF) != 0;
                        fin |= (f ? 1u : 0u) << j;
                        if (f) ring[(R + t + kXT * j) & kMask] = (uint8_t)pp[j];
                        pv[j] = f ? FIN : pp[j];
                        ptr[t + kXT * j] = pp[j];
                    }
                }
                pend &= ~fin;
            }
            if (pend) jflag[it % 3u] = 1u;
            if (t == 0) jflag[(it + 1u) % 3u] = 0u;
            LB_HASH(R, kHashRound)
#ifdef S3HC_LBPROF
            lbp[11] += __builtin_amdgcn_s_memtime() - tb1;
#endif
            LB_SYNC();
            LB_ADD(8, 1);
            if (!jflag[it % 3u]) break;
        }
#if S3HC_LB_OWNFUSE
        // the halves the rounds did not reach (fewer than three rounds)
        if (q + 1 < nsteps && os < 2) {
            if (os == 0) {
                om4 = ((const uint4*)marks)[t];
                oinc = lb_own1(om4, shm);
                LB_SYNC();
            }
            ((uint4*)marks)[t] = lb_own2(om4, oinc, shm);
            os = 2;
            own_sync = true;
        }
#endif
        LB_T(5);
#if S3HC_LB_XBAR
        // every byte of the step is final in the ring (the rounds' last barrier): publish it
        if (t == 0)
            __hip_atomic_store(&x_final, R + kLbStep < size ? R + kLbStep : size, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
#endif
        // flush the step (thread t: dwords t and t + kXT of the step)
        if (dec) {
            const bool al = (((uintptr_t)(ob + R)) & 3u) == 0;
#pragma unroll
            for (uint32_t h = 0; h < 2; ++h) {
                const uint32_t x0 = R + 4u * (t + kXT * h);
                const uint32_t v4 = *(const uint32_t*)(ring + (x0 & kMask));
                if (al && x0 + 4u <= size) {
                    *(uint32_t*)(ob + x0) = v4;
                } else {
#pragma unroll
                    for (uint32_t j = 0; j < 4; ++j)
                        if (x0 + j < size) ob[x0 + j] = (uint8_t)(v4 >> (8 * j));
                }
            }
        }
        LB_T(6);
    }
#undef LB_SYNC
#if !S3HC_LB_XBAR
    // every step is flushed: the hashing wave finishes the stripes, the tail and the avalanche
    __syncthreads();
    LB_HASH(size, hns)
#ifndef S3HC_LB_NOHASH
    if (!dec) {
        const int qb = lane & ~3;
        const uint32_t v1 = __shfl(hacc, qb), v2 = __shfl(hacc, qb + 1), v3 = __shfl(hacc, qb + 2),
                       v4 = __shfl(hacc, qb + 3);
        if (lane == 0) {
            uint32_t h = size >= 16 ? xh_rotl(v1, 1) + xh_rotl(v2, 7) + xh_rotl(v3, 12) + xh_rotl(v4, 18) : XH5;
            h += size;
            uint32_t p = hns * 16u;
            for (; p + 4u <= size; p += 4u) h = xh_rotl(h + *(const u32_unaligned*)(ob + p) * XH3, 17) * XH4;
            for (; p < size; ++p) h = xh_rotl(h + (uint32_t)ob[p] * XH5, 11) * XH1;
            h ^= h >> 15;
            h *= XH2;
            h ^= h >> 13;
            h *= XH3;
            h ^= h >> 16;
            A.blk_hash[B.blk] = (1ull << 32) | h;
        }
    }
#endif
#endif  // !S3HC_LB_XBAR
#ifdef S3HC_LBPROF
    if (t == 0)
        for (int k = 0; k < 12; ++k) atomicAdd(&g_lbprof[k], (unsigned long long)lbp[k]);
#endif
}

#undef LB_T
#undef LB_ADD
#undef LB_HASH
#undef LB_STEP_SEQS
#undef LB_PREFETCH
#undef LB_PUT
#undef LB_INSTALL

// ---------------------------------------------------------------- spread execution
// k_lb_run writes a block with ONE workgroup, step after step: right for a batch that gives every
// CU a block, but one reference cache file (a 1 MiB frame = one block) then keeps 1 of 256 CUs
// busy for 137 serial steps. With few blocks the output is instead cut into tiles of kLbStep
// bytes that are all decoded at once, by as many workgroups as the chip holds:
//
//   k_lbw_plan    (1 workgroup) P positions and tiles of the blocks that fit P (wcap);
//   k_lbw_init    per tile: every byte gets its value (literal) or its source (matches: the
//                 first period of an overlapping copy), chains inside the tile are jumped in LDS;
//                 final bytes are stored, every other byte leaves a pointer to a byte of an
//                 earlier tile in P (global positions);
//   k_lbw_round   x kLbwRounds: pointer jumping over P (each pending byte reads its source's
//                 entry: final -> that source is its root; resolved -> take the root; else jump),
//                 up to kLbwHops hops per launch. Entries only move along their chain, so reading
//                 a value another workgroup is replacing in the same launch is harmless; roots are
//                 always bytes k_lbw_init stored (earlier launch: visible). A launch with nothing
//                 pending returns at once;
//   k_lbw_gather  every pending byte copies its root's byte (walking what the rounds left: every
//                 pointer goes to a smaller position, so every chain ends).
namespace lb {
constexpr uint32_t PFIN = 0xFFFFFFFFu;  // P: the byte in dst is final
constexpr uint32_t PRES = 0x80000000u;  // P: flag of a resolved entry (1 << 31 | root); PFIN has it too
constexpr uint32_t LOUT = 0x80000000u;  // k_lbw_init LDS pointer: source before the tile (P position < 2^30)
constexpr uint32_t LFIN = 0x40000000u;  // k_lbw_init LDS entry of a final byte: LFIN | value
}  // namespace lb

__global__ __launch_bounds__(1024) void k_lbw_plan(LbArgs A, uint32_t* __restrict__ blk_out, int32_t* __restrict__ blk_status) {
    using namespace lb;
    __shared__ uint64_t shs[16];
    __shared__ uint32_t sht[16];
    __shared__ uint64_t cpos;
    __shared__ uint32_t ctile;
    const uint32_t t = threadIdx.x;
    if (t < kLbwRounds + 2) A.ctl->rflag[t] = 0u;
    if (t == 0) { cpos = 0; ctile = 0; }
    __syncthreads();
    const uint32_t nlb = A.ctl->nlb;
    // blocks of frames that allow more than 64 KiB spread (small blocks gain little from it and
    // lose the step loop's overlap with other queues), and only when there are few of them
    uint32_t nbig = 0;
    for (uint32_t i = t; i < nlb; i += 1024) nbig += A.lbt[i].limit > kLbwMinLimit ? 1u : 0u;
    uint32_t totbig;
    (void)wg_excl_add<uint32_t, 16>(nbig, sht, totbig);
    const bool few = totbig <= kLbwMaxBlocks;
    for (uint32_t base = 0; base < nlb; base += 1024) {
        const uint32_t i = base + t;
        // (k_lb_fin's work, done here when the spread execution runs)
        uint32_t fsize = 0, fstat = S3HC_CORRUPT;
        if (i < nlb) fstat = lb_fin_block(A, i, blk_out, blk_status, &fsize);
        const bool ok = few && i < nlb && fstat == S3HC_OK && fsize > 0 && A.lbt[i].limit > kLbwMinLimit;
        const uint32_t size = ok ? fsize : 0u;
        uint64_t tots;
        uint32_t tott;
        // positions grow with the block index, so the spread blocks are a prefix of the decodable ones
        const uint64_t pp = wg_excl_add<uint64_t, 16>((uint64_t)size, shs, tots) + cpos;
        const bool wide = ok && pp + size <= A.wcap;
        const uint32_t nt = wide ? (size + kLbStep - 1) / kLbStep : 0u;
        const uint32_t tp = wg_excl_add<uint32_t, 16>(nt, sht, tott) + ctile;
        if (i < nlb) {
            A.wbase[i] = wide ? (uint32_t)pp : NONE;
            A.wtile0[i] = tp;
        }
        __syncthreads();
        if (t == 0) { cpos += tots; ctile += tott; }
        __syncthreads();
    }
    if (t == 0) A.ctl->ntiles = ctile;
}

// LB block holding tile T: the last block whose first tile is <= T (blocks without tiles repeat
// their successor's first tile and are skipped by that rule)
__device__ __forceinline__ uint32_t lbw_block(const LbArgs& A, uint32_t nlb, uint32_t T) {
    uint32_t lo = 0, hi = nlb;
    while (hi - lo > 1u) {
        const uint32_t mid = (lo + hi) >> 1;
        if (A.wtile0[mid] <= T) lo = mid;
        else hi = mid;
    }
    return lo;
}

__global__ __launch_bounds__(960) void k_lbw_init(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, LbArgs A) {
    using namespace lb;
    __shared__ __attribute__((aligned(16))) uint16_t marks[kLbStep];
    __shared__ __attribute__((aligned(16))) uint32_t sqp[kMaxSeqS * 4];  // the tile's sequences, then its pointers
    __shared__ uint16_t so[kMaxSeqS];
    __shared__ __attribute__((aligned(16))) uint8_t val[kLbStep];
    __shared__ __attribute__((aligned(16))) uint32_t shm[16];
    __shared__ uint32_t jflag[3];
    static_assert(kLbStep <= kMaxSeqS * 4, "pointers fit the sequence table's space");
    uint4* sq = (uint4*)sqp;
    uint32_t* ptr = sqp;
    const uint32_t t = threadIdx.x;
    const uint32_t ntiles = A.ctl->ntiles, nlb = A.ctl->nlb;
    for (uint32_t T = blockIdx.x; T < ntiles; T += gridDim.x) {
        const uint32_t i = lbw_block(A, nlb, T);
        const uint32_t q = T - A.wtile0[i];
        const LbBlock B = A.lbt[i];
        const uint32_t size = A.lb_size[i], wb = A.wbase[i], tok0 = A.lb_tok0[i], ntok = A.lb_ntok[i];
        const uint32_t nsteps = (size + kLbStep - 1) / kLbStep;
        const uint32_t R = q * kLbStep;
        const uint8_t* g = src + B.src_off;
        uint8_t* ob = dst + B.dst_off;
        const uint32_t s0 = A.rfirst[(size_t)i * kLbMaxSteps + q];
        const uint32_t s1 = q + 1 < nsteps ? A.rfirst[(size_t)i * kLbMaxSteps + q + 1] + 1u : ntok;
        const uint32_t ns = s1 - s0 < kMaxSeqS ? s1 - s0 : kMaxSeqS;
        ((uint4*)marks)[t] = make_uint4(0, 0, 0, 0);  // kLbStep u16 = 960 x 16 B
        __syncthreads();
        for (uint32_t j = t; j < ns; j += kXT) {
            const uint4 e = A.seq4[tok0 + s0 + j];
            sq[j] = e;
            so[j] = A.seqoff[tok0 + s0 + j];
            const uint32_t rel = e.x > R ? e.x - R : 0u;
            if (rel < kLbStep && (j == 0 || e.x > R)) marks[rel] = (uint16_t)(j + 1u);
        }
        __syncthreads();
        // owner of each byte: running max of the start marks (thread t: bytes 8t .. 8t+7)
        const uint4 own = lb_owners(((const uint4*)marks)[t], shm);
        ((uint4*)marks)[t] = own;
        __syncthreads();
        // classify (thread t: bytes t + kXT*j): literal (input address) or match source, taken in
        // the first period of an overlapping copy; sources inside the tile become LDS pointers,
        // sources before it P positions
        uint32_t la[kXPer], pv[kXPer];
        uint32_t litm = 0;
#pragma unroll
        for (uint32_t j = 0; j < kXPer; ++j) {
            const uint32_t l = t + kXT * j;
            const uint32_t x = R + l;
            pv[j] = FIN;
            la[j] = 0;
            if (x < size) {
                const uint32_t k = marks[l] - 1u;
                const uint4 e = sq[k];
                const uint32_t rel = x - e.x;
                if (rel < e.z) {
                    la[j] = e.y + rel;
                    litm |= 1u << j;
                } else {
                    const uint32_t off = so[k];
                    const uint32_t ee = rel - e.z;  // position inside the match
                    const uint32_t y = ee >= off ? e.x + e.z - off + ee % off : x - off;
                    pv[j] = y >= R ? y - R : (LOUT | (wb + y));
                }
            }
        }
        uint32_t lv[kXPer];
#pragma unroll
        for (uint32_t j = 0; j < kXPer; ++j) lv[j] = g[(litm >> j) & 1u ? la[j] : 0u];
        __syncthreads();  // every read of sq is done before the pointers overwrite it
#pragma unroll
        for (uint32_t j = 0; j < kXPer; ++j) {
            const uint32_t l = t + kXT * j;
            val[l] = (uint8_t)((litm >> j) & 1u ? lv[j] : 0u);
            ptr[l] = pv[j] == FIN ? (LFIN | lv[j]) : pv[j];  // a final byte's entry carries its value
        }
        if (t == 0) jflag[0] = 0u;
        __syncthreads();
        // chains inside the tile (as in k_lb_run): a final source gives the value (its entry is
        // LFIN | byte), a source that points before the tile hands over its P position, a pending
        // one is jumped over; two hops per round
        uint32_t pend = 0;
#pragma unroll
        for (uint32_t j = 0; j < kXPer; ++j) pend |= (!(pv[j] & LOUT) ? 1u : 0u) << j;
        for (uint32_t it = 0; it < 16; ++it) {
            for (uint32_t h = 0; h < kJumpHops && pend; ++h) {
                uint32_t pp[kXPer];
#pragma unroll
                for (uint32_t j = 0; j < kXPer; ++j) pp[j] = (pend >> j) & 1u ? ptr[pv[j]] : 0u;
                uint32_t done = 0;
#pragma unroll
                for (uint32_t j = 0; j < kXPer; ++j) {
                    if ((pend >> j) & 1u) {
                        const bool f = (pp[j] & LFIN) != 0;
                        if (f) val[t + kXT * j] = (uint8_t)pp[j];
                        pv[j] = f ? FIN : pp[j];
                        done |= ((pv[j] & LOUT) ? 1u : 0u) << j;
                        ptr[t + kXT * j] = pp[j];
                    }
                }
                pend &= ~done;
            }
            if (pend) jflag[it % 3u] = 1u;
            if (t == 0) jflag[(it + 1u) % 3u] = 0u;
            __syncthreads();
            if (!jflag[it % 3u]) break;
        }
        // store: final bytes (coalesced dwords from LDS), every byte's P entry
        const bool al = (((uintptr_t)(ob + R)) & 3u) == 0;
#pragma unroll
        for (uint32_t h = 0; h < 2; ++h) {
            const uint32_t l0 = 4u * (t + kXT * h);
            const uint32_t x0 = R + l0;
            const uint32_t v4 = *(const uint32_t*)(val + l0);
            if (al && x0 + 4u <= size) {
                *(uint32_t*)(ob + x0) = v4;
            } else {
#pragma unroll
                for (uint32_t j = 0; j < 4; ++j)
                    if (x0 + j < size) ob[x0 + j] = (uint8_t)(v4 >> (8 * j));
            }
        }
        bool out = false;
#pragma unroll
        for (uint32_t j = 0; j < kXPer; ++j) {
            const uint32_t x = R + t + kXT * j;
            if (x < size) {
                const bool o = pv[j] != FIN;
                out |= o;
                A.P[wb + x] = o ? (pv[j] & ~LOUT) : PFIN;
            }
        }
        const int po = __syncthreads_or(out);  // also: every read of val/marks of this tile is done
        if (t == 0) {
            A.tpend[T] = po ? 1 : 0;
            A.tinit[T] = po ? 1 : 0;
            if (po) atomicAdd(&A.ctl->rflag[0], 1u);
        }
    }
}

__global__ __launch_bounds__(960) void k_lbw_round(LbArgs A, uint32_t r) {
    using namespace lb;
    if (!A.ctl->rflag[r]) return;
    const uint32_t t = threadIdx.x;
    const uint32_t ntiles = A.ctl->ntiles, nlb = A.ctl->nlb;
    uint32_t npend = 0;  // tiles of this workgroup still pending after the launch
    for (uint32_t T = blockIdx.x; T < ntiles; T += gridDim.x) {
        if (!A.tpend[T]) continue;
        const uint32_t i = lbw_block(A, nlb, T);
        const uint32_t q = T - A.wtile0[i];
        const uint32_t size = A.lb_size[i], wb = A.wbase[i];
        const uint32_t R = q * kLbStep;
        uint32_t v[kXPer];
        uint32_t pend = 0;
#pragma unroll
        for (uint32_t j = 0; j < kXPer; ++j) {
            const uint32_t x = R + t + kXT * j;
            v[j] = x < size ? A.P[wb + x] : PFIN;
            pend |= ((v[j] & PRES) ? 0u : 1u) << j;
        }
        const uint32_t touched = pend;
        // up to kLbwHops hops per launch (entries read here may already be this launch's)
        for (uint32_t h = 0; h < kLbwHops && pend; ++h) {
            uint32_t w[kXPer];
#pragma unroll
            for (uint32_t j = 0; j < kXPer; ++j) w[j] = (pend >> j) & 1u ? A.P[v[j]] : 0u;
#pragma unroll
            for (uint32_t j = 0; j < kXPer; ++j) {
                if ((pend >> j) & 1u) {
                    v[j] = w[j] == PFIN ? (v[j] | PRES) : w[j];
                    if (v[j] & PRES) pend &= ~(1u << j);
                }
            }
        }
#pragma unroll
        for (uint32_t j = 0; j < kXPer; ++j)
            if ((touched >> j) & 1u) A.P[wb + R + t + kXT * j] = v[j];
        const int ps = __syncthreads_or(pend != 0);
        if (t == 0) A.tpend[T] = ps ? 1 : 0;
        npend += ps ? 1u : 0u;
    }
    if (t == 0 && npend) atomicAdd(&A.ctl->rflag[r + 1], npend);
}

__global__ __launch_bounds__(960) void k_lbw_gather(uint8_t* __restrict__ dst, LbArgs A) {
    using namespace lb;
    const uint32_t t = threadIdx.x;
    const uint32_t ntiles = A.ctl->ntiles, nlb = A.ctl->nlb;
    for (uint32_t T = blockIdx.x; T < ntiles; T += gridDim.x) {
        if (!A.tinit[T]) continue;
        const uint32_t i = lbw_block(A, nlb, T);
        const uint32_t q = T - A.wtile0[i];
        const uint32_t size = A.lb_size[i], wb = A.wbase[i];
        uint8_t* ob = dst + A.lbt[i].dst_off;
        const uint32_t R = q * kLbStep;
        uint32_t v[kXPer], b[kXPer];
#pragma unroll
        for (uint32_t j = 0; j < kXPer; ++j) {
            const uint32_t x = R + t + kXT * j;
            v[j] = x < size ? A.P[wb + x] : PFIN;
        }
        // a chain the rounds did not finish (only for chains far longer than data holds) is
        // walked here: P no longer changes, and every pointer goes to a smaller position
#pragma unroll
        for (uint32_t j = 0; j < kXPer; ++j) {
            while (!(v[j] & PRES)) {
                const uint32_t w = A.P[v[j]];
                v[j] = w == PFIN ? (v[j] | PRES) : w;
            }
        }
        // roots: 1 << 31 | position of a byte k_lbw_init stored
#pragma unroll
        for (uint32_t j = 0; j < kXPer; ++j) b[j] = v[j] != PFIN ? ob[(v[j] & ~PRES) - wb] : 0u;
#pragma unroll
        for (uint32_t j = 0; j < kXPer; ++j)
            if (v[j] != PFIN) ob[R + t + kXT * j] = (uint8_t)b[j];
    }
}

// ================================================================ launchers
static inline uint32_t cdiv_lb(uint64_t a, uint64_t b) { return (uint32_t)((a + b - 1) / b); }
hipError_t launch_scan2(const uint32_t* in0, const uint32_t* in1, uint32_t n, uint64_t* out0, uint64_t* out1,
                        uint64_t* total, hipStream_t st);

// Parse stage: classify the units, tokenize, build the sequence table, statuses and sizes of
// the taken blocks. Must precede k_decode_units (it reads unit_lb).
hipError_t launch_lb_parse(const LbArgs& A, const uint8_t* src, const DecBlock* blk, const DecUnit* units,
                           uint32_t nunits, const uint64_t* ucount, uint32_t* blk_out, int32_t* blk_status,
                           hipStream_t st) {
    hipLaunchKernelGGL(k_lb_classify, dim3(1), dim3(1024), 0, st, blk, units, nunits, ucount, A);
    hipLaunchKernelGGL(k_lb_gran, dim3(A.chunk_cap), dim3(lb::kGpc), 0, st, src, A);
#if S3HC_LB_TOKV2
    hipLaunchKernelGGL(k_lbt_walk, dim3(A.chunk_cap), dim3(lb::kWT), 0, st, src, A);
    hipLaunchKernelGGL(k_lbt_entry, dim3(cdiv_lb(A.lb_cap, 64)), dim3(64), 0, st, src, A);
    hipLaunchKernelGGL(k_lbt_mark, dim3(A.chunk_cap), dim3(lb::kWT), 0, st, src, A);
#else
    hipLaunchKernelGGL(k_lb_exit, dim3(A.chunk_cap), dim3(lb::kT), 0, st, src, A);
    hipLaunchKernelGGL(k_lb_entry, dim3(cdiv_lb(A.lb_cap, 64)), dim3(64), 0, st, A);
    hipLaunchKernelGGL(k_lb_mark, dim3(A.chunk_cap), dim3(lb::kT), 0, st, src, A);
#endif
    hipError_t e = launch_scan2(A.ntok, A.slsum, A.chunk_cap, A.tokbase, A.outbase, A.total, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_lb_seq, dim3(A.chunk_cap), dim3(lb::kSeqT), 0, st, src, A);
    if (!A.wcap)  // (with the spread execution, k_lbw_plan does it)
        hipLaunchKernelGGL(k_lb_fin, dim3(cdiv_lb(A.lb_cap, 256)), dim3(256), 0, st, A, blk_out, blk_status);
    return hipGetLastError();
}

// Execute stage: one workgroup per taken block.
hipError_t launch_lb_exec(const LbArgs& A, const uint8_t* src, uint8_t* dst, uint32_t* blk_out, int32_t* blk_status,
                          hipStream_t st) {
    if (A.wcap) {  // spread execution of the blocks that fit P, then the step loop for the rest
        const uint32_t tiles = A.tile_cap;
        hipLaunchKernelGGL(k_lbw_plan, dim3(1), dim3(1024), 0, st, A, blk_out, blk_status);
        hipLaunchKernelGGL(k_lbw_init, dim3(tiles < 512u ? tiles : 512u), dim3(lb::kXT), 0, st, src, dst, A);
        // S3HC_LBW_ROUNDS (tests): fewer launches, so k_lbw_gather walks long chains itself
        uint32_t rounds = kLbwRounds;
        if (knob(KN_LBW_ROUNDS) >= 0) rounds = std::min<uint32_t>(rounds, (uint32_t)knob(KN_LBW_ROUNDS));
        for (uint32_t r = 0; r < rounds; ++r)
            hipLaunchKernelGGL(k_lbw_round, dim3(tiles < 512u ? tiles : 512u), dim3(lb::kXT), 0, st, A, r);
        hipLaunchKernelGGL(k_lbw_gather, dim3(tiles < 1024u ? tiles : 1024u), dim3(lb::kXT), 0, st, dst, A);
    }
    if (!A.all_spread) hipLaunchKernelGGL(k_lb_run, dim3(A.lb_cap), dim3(lb::kXWG), 0, st, src, dst, A);
    return hipGetLastError();
}
}  // namespace s3hc

#ifdef S3HC_LBPROF
extern "C" int s3hc_diag_lbprof(unsigned long long* out, int reset) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(s3hc::g_lbprof), sizeof(unsigned long long) * 32) != hipSuccess) return -1;
    if (reset) {
        unsigned long long z[32] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(s3hc::g_lbprof), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#endif
