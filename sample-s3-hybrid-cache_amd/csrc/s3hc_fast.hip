// s3hc_fast.hip — the 64 KiB-block LZ4 decode path and the small-batch decoders
// (§4f, §4g). Compiled inside s3hc_kernels.hip (one translation unit: k_djump runs its per-unit
// decoder and frame close), never on its own.
//
// lz4_flex's FrameDecoder (compression.rs:479-480) decodes a block by one serial walk: token,
// literal run, offset, match, next token. Here that walk is split in two kernels:
//
//   k_dtok   token index. One 256-thread workgroup per block stages the compressed block in LDS
//            and cuts it into 256 segments. Every thread walks the token chain from the start of
//            its segment as if a token began there (speculatively), marking the positions it
//            visits in a bitmap; past its segment's end it keeps walking until it lands on a
//            position another thread marked (LZ4 token chains merge after a few hops: a chain is
//            a function of its position). The true chain is the first thread's walk, then the
//            walk it merged into, and so on: those "merge into" links form a list over the
//            segments that pointer doubling resolves in 8 steps. The true tokens are then
//            counted (bitmap popcounts), scanned, validated against every lz4_flex bound (literal
//            and match lengths against the block limit and the caller's capacity, offsets against
//            the bytes produced) and their positions written to a pool.
//   k_dexec  executor (one wave per block): 64 sequences at a time, one per lane.
//
// A block the fast path does not take (stored, larger than kFastMaxC compressed bytes, part of a
// multi-block unit, or failing any check) is left to the per-unit decoder (k_decode_pe), which
// also reports its exact status; the fast path only ever produces correct output for valid
// blocks, so its results are the per-unit decoder's by construction.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "s3hc_plan.hpp"
#include "s3hc_lz4.h"

// Phase timers of diagnostic builds only (S3HC_DIAG_LEVEL 10): per-wave s_memtime sums into
// g_fprof, read back with s3hc_diag_fprof. Compiled out of the shipped library.
#if defined(S3HC_DIAG_LEVEL) && S3HC_DIAG_LEVEL == 10
#define FPROF 1
#define FP_NOW() __builtin_amdgcn_s_memtime()
#define FP_ADD(k, v) atomicAdd(&s3hc::g_fprof[k], (unsigned long long)(v))
#else
#define FP_NOW() 0ull
#define FP_ADD(k, v) ((void)0)
#endif

namespace s3hc {
#ifdef FPROF
__device__ unsigned long long g_fprof[32];
#endif
#if defined(FPROF) || (defined(S3HC_UPROF) && S3HC_UPROF)
#define UPROF 1
// per executor unit (u < 8192): start, end (s_memrealtime, 100 MHz), HW_ID, XCC_ID | sweeps << 8 | windows << 32
__device__ unsigned long long g_uprof[8192][4];
#endif
namespace fst {
constexpr uint32_t kMaxC = kFastMaxC;
#ifndef S3HC_DTOK_TT
#define S3HC_DTOK_TT 256
#endif
#ifndef S3HC_HOP2  // 1: k_dtok parses tokens with hop2 (branch-light), 0: hop
#define S3HC_HOP2 1
#endif
#if S3HC_HOP2
#define S3HC_HOPF hop2
#else
#define S3HC_HOPF hop
#endif
#ifndef S3HC_DTOK_SKIP  // diagnostic builds only (timing, output wrong): 1 no record stores, 2 no token parse in the record pass
#define S3HC_DTOK_SKIP 0
#endif
#ifndef S3HC_DTOK_BAL  // 1: records by sequence rank, 0: by bitmap words
#define S3HC_DTOK_BAL 1
#endif
constexpr uint32_t kTT = S3HC_DTOK_TT;         // k_dtok threads = speculative segments per block
constexpr uint32_t kStage = kMaxC + 64;        // staged block: 16-B alignment slack + zero read-ahead
constexpr uint32_t kBitW = kMaxC / 32;         // bitmap words, one bit per compressed position
constexpr uint32_t END = 0xFFFFFFFEu;          // chain ended with the block's last sequence
constexpr uint32_t DEAD = 0xFFFFFFFFu;         // malformed token (or a walk that gave up)
constexpr uint32_t kOvfCap = 4096;             // hops a walk past its segment may take before giving up
static_assert(kTT == 256 || kTT == 512 || kTT == 1024, "k_dtok: 4, 8 or 16 waves");
static_assert(kBitW <= 4 * 256, "k_dtok: four bitmap words per thread cover the block");
constexpr uint32_t kMEnd = 0xFFFEu, kMBad = 0xFFFFu;  // u16 merge codes (positions are < kMaxC)
}  // namespace fst

namespace {
__device__ __forceinline__ uint32_t umin_(uint32_t a, uint32_t b) { return a < b ? a : b; }
__device__ __forceinline__ uint32_t umax_(uint32_t a, uint32_t b) { return a > b ? a : b; }

// 4 bytes at LDS byte offset i (two aligned dword reads + v_alignbyte)
__device__ __forceinline__ uint32_t st32(const uint8_t* st, uint32_t i) {
    const uint32_t* w = (const uint32_t*)(st + (i & ~3u));
    return __builtin_amdgcn_alignbyte(w[1], w[0], i & 3u);
}

// Remainder of a length-extension run at block byte q (the inline decode already consumed two
// bytes of 255): adds the run, advances q past it; q = C + 1 when the run reaches the end.
__device__ uint32_t ext_tail(const uint8_t* st, uint32_t mis, uint32_t& q, uint32_t C) {
    uint32_t acc = 0;
    for (;;) {
        if (q >= C) {
            q = C + 1;
            return acc;
        }
        const uint32_t e = st[q + mis];
        ++q;
        acc += e;
        if (e != 255u) return acc;
    }
}

struct Tok {
    uint32_t nxt;  // next token position, END (this is the last sequence) or DEAD (malformed)
    uint32_t ll, off, ml;
};

// One token of the staged block at position p (lz4_flex decompress_internal's parse: literal
// length with 255-runs, literals, 2-byte offset, match length with 255-runs). A block must end
// right after a literal run; a run, an offset or literals reaching past the end are malformed.
__device__ __forceinline__ Tok hop(const uint8_t* st, uint32_t mis, uint32_t p, uint32_t C) {
    Tok T;
    T.off = 0;
    T.ml = 0;
    const uint32_t w0 = st32(st, p + mis);
    const uint32_t t = w0 & 0xFFu;
    uint32_t L = t >> 4, q = p + 1;
    if (L == 15u) {
        const uint32_t e1 = (w0 >> 8) & 0xFFu;
        L += e1;
        ++q;
        if (e1 == 255u) {
            const uint32_t e2 = (w0 >> 16) & 0xFFu;
            L += e2;
            ++q;
            if (e2 == 255u) L += ext_tail(st, mis, q, C);
        }
    }
    T.ll = L;
    if (q > C || L > C - q) {  // run past the end / literals past the end
        T.nxt = fst::DEAD;
        return T;
    }
    const uint32_t mp = q + L;
    if (mp == C) {  // last sequence: literals only
        T.nxt = fst::END;
        return T;
    }
    if (C - mp < 2) {
        T.nxt = fst::DEAD;
        return T;
    }
    const uint32_t w1 = st32(st, mp + mis);
    T.off = w1 & 0xFFFFu;
    uint32_t M = (t & 15u) + 4u, q2 = mp + 2;
    if ((t & 15u) == 15u) {
        const uint32_t f1 = (w1 >> 16) & 0xFFu;
        M += f1;
        ++q2;
        if (f1 == 255u) {
            const uint32_t f2 = w1 >> 24;
            M += f2;
            ++q2;
            if (f2 == 255u) M += ext_tail(st, mis, q2, C);
        }
    }
    T.ml = M;
    T.nxt = q2 >= C ? fst::DEAD : q2;  // a run past the end, or no token after a match
    return T;
}

// The same token parse with the common cases branch-free (one length-extension byte per field as
// selects; two or more extension bytes, rare, in a branch) and the verdicts computed last as
// selects: the same (nxt, ll, off, ml) as hop() for every input (an offset word past the block is
// read at a clamped address and ignored: the verdict is DEAD or END there).
__device__ __forceinline__ Tok hop2(const uint8_t* st, uint32_t mis, uint32_t p, uint32_t C) {
    Tok T;
    const uint32_t w0 = st32(st, p + mis);
    const uint32_t t = w0 & 0xFFu;
    uint32_t L = t >> 4, q = p + 1u;
    const uint32_t b1 = (w0 >> 8) & 0xFFu;
    const bool x1 = L == 15u;
    L += x1 ? b1 : 0u;
    q += x1 ? 1u : 0u;
    if (x1 && b1 == 255u) {  // rare: a second extension byte (and more)
        const uint32_t b2 = (w0 >> 16) & 0xFFu;
        L += b2;
        ++q;
        if (b2 == 255u) L += ext_tail(st, mis, q, C);
    }
    const uint32_t mp = q + L;
    const uint32_t w1 = st32(st, umin_(mp, C) + mis);
    uint32_t M = (t & 15u) + 4u, q2 = mp + 2u;
    const uint32_t f1 = (w1 >> 16) & 0xFFu;
    const bool x2 = (t & 15u) == 15u;
    M += x2 ? f1 : 0u;
    q2 += x2 ? 1u : 0u;
    if (x2 && f1 == 255u && mp <= C) {  // rare
        const uint32_t f2 = w1 >> 24;
        M += f2;
        ++q2;
        if (f2 == 255u) M += ext_tail(st, mis, q2, C);
    }
    const bool dead_lit = q > C || L > C - q;
    const bool end = mp == C;
    T.ll = L;
    T.off = dead_lit || end ? 0u : w1 & 0xFFFFu;
    T.ml = dead_lit || end ? 0u : M;
    T.nxt = dead_lit ? fst::DEAD : (end ? fst::END : ((C - mp < 2u || q2 >= C) ? fst::DEAD : q2));
    return T;
}

// inclusive wave sum by DPP row shifts and row broadcasts (lanes without a source read 0; no
// ds_bpermute round trip)
__device__ __forceinline__ uint32_t wave_incl_sum_dpp(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);
    return x;
}
// exclusive scan over the NW waves of a workgroup; *total = sum
template <uint32_t NW>
__device__ __forceinline__ uint32_t wg_excl_scan(uint32_t v, uint32_t* scratch, uint32_t* total) {
    const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
    const uint32_t x = wave_incl_sum_dpp(v);
    if (lane == 63) scratch[w] = x;
    __syncthreads();
    uint32_t before = 0, all = 0;
#pragma unroll
    for (uint32_t k = 0; k < NW; ++k) {
        const uint32_t sk = scratch[k];
        before += k < w ? sk : 0u;
        all += sk;
    }
    *total = all;
    __syncthreads();
    return before + x - v;
}
// two exclusive scans over the workgroup at once (one scratch exchange, two barriers)
template <uint32_t NW>
__device__ __forceinline__ void wg_excl_scan2(uint32_t v, uint32_t u, uint32_t* scratch, uint32_t* ev, uint32_t* eu,
                                              uint32_t* tv, uint32_t* tu) {
    const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
    const uint32_t x = wave_incl_sum_dpp(v), y = wave_incl_sum_dpp(u);
    if (lane == 63) {
        scratch[2 * w] = x;
        scratch[2 * w + 1] = y;
    }
    __syncthreads();
    uint32_t bx = 0, by = 0, ax = 0, ay = 0;
#pragma unroll
    for (uint32_t k = 0; k < NW; ++k) {
        const uint32_t sx = scratch[2 * k], sy = scratch[2 * k + 1];
        bx += k < w ? sx : 0u;
        by += k < w ? sy : 0u;
        ax += sx;
        ay += sy;
    }
    *tv = ax;
    *tu = ay;
    *ev = bx + x - v;
    *eu = by + y - u;
    __syncthreads();
}
}  // namespace

__device__ __forceinline__ void wsync_blk() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ------------------------------------------------------------------ k_dtok
// Returns whether the fast path took unit u (workgroup-uniform); *fo = its (sequences, bytes).
template <uint32_t TT>  // threads of the workgroup = speculative segments per block (256, 512 or 1024)
__device__ __forceinline__ bool dtok_unit(const uint32_t u, const uint8_t* __restrict__ src,
                                          const DecBlock* __restrict__ blk, const DecUnit* __restrict__ units,
                                          const uint8_t* __restrict__ unit_lb, const FastArgs& a,
                                          uint32_t maxc, FastUnit* fo) {
    using namespace fst;
    static_assert(TT == 256 || TT == 512 || TT == 1024, "dtok_unit: 4, 8 or 16 waves");
    constexpr uint32_t kLv = TT == 1024 ? 10 : (TT == 512 ? 9 : 8);  // doubling levels: chains over <= TT segments
    constexpr uint32_t kTermEnd = TT, kTermBad = TT + 1;
    // the staged block and the token bitmap live in dynamic LDS sized to the launch's largest
    // compressed block (fast_lds_bytes): config 2's ~26 KB blocks fit five workgroups per CU
    // instead of four at the 32 KiB maximum
    extern __shared__ __attribute__((aligned(16))) uint8_t dsm[];
    uint8_t* stage = dsm;
    uint32_t* bits = (uint32_t*)(dsm + fast_stage_bytes(maxc));
    __shared__ uint16_t svfrom[TT];   // per segment on the true chain: its first true token (else M_BAD)
    __shared__ uint16_t J[2][TT + 2]; // succ^(2^k) per segment, ping-pong; TT / TT + 1 are terminals
    __shared__ uint8_t reach[TT + 2]; // segment is on the true chain
    __shared__ uint32_t scr[16];
    __shared__ uint32_t sflag[4];      // [0] terminal of the chain, [1] failure, [2] pool base
    const uint32_t g = threadIdx.x;
    const DecUnit U = units[u];
    bool take = U.n == 1 && !(unit_lb && unit_lb[u]);
    DecBlock B;
    if (take) {
        B = blk[U.first];
        // (blocks of frames allowing at most 64 KiB: a sequence record holds ll < 2^17 and
        // ml - 4 < 2^16; larger blocks take the large-block path or the per-unit decoder)
        take = !(B.flags & DB_STORED) && B.csize >= 1u && B.csize <= maxc && B.limit <= 65536u;
    }
    // a unit the fast path leaves: no hash for the frame close (large blocks: the large-block path's)
    auto leave = [&]() {
        if (g == 0) {
            a.unit_fast[u] = 0;
            if (a.bh && U.n == 1 && !(unit_lb && unit_lb[u])) a.bh[U.first] = 0;
        }
    };
    if (!take) {
        leave();
        return false;
    }
    const uint32_t C = B.csize;
    [[maybe_unused]] const uint64_t tp0 = FP_NOW();
    // ---- stage the block: aligned 16-byte loads (never outside the 16-byte granules holding
    // block bytes), four in flight per thread before their LDS stores
    const uint8_t* in = src + B.src_off;
    const uint32_t mis = (uint32_t)((uintptr_t)in & 15u);
    {
        // (mis + C + 15) / 16 <= 2050 granules: at most 9 (256 threads) or 5 (512) per thread,
        // all loads in flight at once
        const uint4* gw = (const uint4*)(in - mis);
        const uint32_t nv = (mis + C + 15u) >> 4;
        static_assert((kMaxC + 30u) / 16u <= (TT == 256 ? 9u : 5u) * TT, "staging covers the largest block");
        uint4 v0, v1, v2, v3, v4, v5, v6, v7, v8;
#define S3HC_LDG(i, v) if (g + (i) * TT < nv) v = gw[g + (i) * TT];
#define S3HC_STS(i, v) if (g + (i) * TT < nv) ((uint4*)stage)[g + (i) * TT] = v;
        S3HC_LDG(0, v0) S3HC_LDG(1, v1) S3HC_LDG(2, v2) S3HC_LDG(3, v3) S3HC_LDG(4, v4)
        if (TT == 256) { S3HC_LDG(5, v5) S3HC_LDG(6, v6) S3HC_LDG(7, v7) S3HC_LDG(8, v8) }
        S3HC_STS(0, v0) S3HC_STS(1, v1) S3HC_STS(2, v2) S3HC_STS(3, v3) S3HC_STS(4, v4)
        if (TT == 256) { S3HC_STS(5, v5) S3HC_STS(6, v6) S3HC_STS(7, v7) S3HC_STS(8, v8) }
#undef S3HC_LDG
#undef S3HC_STS
        for (uint32_t k = g; k < (C + 31u) / 32u; k += TT) bits[k] = 0u;
        reach[g] = g == 0 ? 1 : 0;
        if (g == 0) {
            sflag[0] = kTermBad;
            sflag[1] = 0u;
        }
    }
    __syncthreads();
    if (g < 48u) stage[mis + C + g] = 0;  // read-ahead past the block reads zeros
    __syncthreads();

    [[maybe_unused]] const uint64_t tp1 = FP_NOW();
    // ---- walk 1: from the start of my segment to its end, marking every position visited
    const uint32_t segL = (C + TT - 1u) / TT;
    const uint32_t s0 = umin_(g * segL, C), s1 = umin_(s0 + segL, C);
    uint32_t p = s0;
    while (p < s1) {
        atomicOr(&bits[p >> 5], 1u << (p & 31u));
        p = S3HC_HOPF(stage, mis, p, C).nxt;
    }
    const uint32_t x = s0 < s1 ? p : DEAD;
    __syncthreads();
    [[maybe_unused]] const uint64_t tp2 = FP_NOW();
    // ---- walk 2: past the segment until the chain lands on a marked position (merge)
    uint32_t m = x, ovf = 0;
    while (m < C) {
        if ((bits[m >> 5] >> (m & 31u)) & 1u) break;
        if (ovf == kOvfCap) {
            m = DEAD;
            break;
        }
        m = S3HC_HOPF(stage, mis, m, C).nxt;
        ++ovf;
    }
#ifdef FPROF
    {
        uint32_t mx = ovf;
        for (int d = 32; d >= 1; d >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, d, 64));
        if ((g & 63u) == 0) FP_ADD(10, mx);
    }
#endif
    const uint32_t smerge = m < C ? m : (m == END ? kMEnd : kMBad);  // where my walk merged
    svfrom[g] = kMBad;
    // successor segment of my walk: the segment of the merge point, or a terminal
    J[0][g] = (uint16_t)(m < C ? m / segL : (m == END ? kTermEnd : kTermBad));
    if (g < 2) {
        J[0][TT + g] = J[1][TT + g] = (uint16_t)(TT + g);
        reach[TT + g] = 0;
    }
    __syncthreads();
    [[maybe_unused]] const uint64_t tp3 = FP_NOW();
    // ---- the true chain: segment 0, then the segment its walk merged into, ... Reachability
    // from segment 0 by doubling: after step k every segment within 2^(k+1) links is marked.
#pragma unroll
    for (uint32_t k = 0; k < kLv; ++k) {
        const uint32_t h = J[k & 1][g];
        if (reach[g]) reach[h] = 1;
        J[(k + 1) & 1][g] = J[k & 1][h];
        __syncthreads();
    }
    // a segment on the chain hands its merge point to its successor (that segment's first true
    // token); the chain's last segment ends it: END, or a malformed / abandoned walk
    if (reach[g]) {
        const uint32_t sm = smerge;
        if (sm < kMEnd) svfrom[sm / segL] = (uint16_t)sm;
        else sflag[0] = sm == kMEnd ? kTermEnd : kTermBad;
    }
    if (g == 0) svfrom[0] = 0;
    __syncthreads();
    if (sflag[0] != kTermEnd) {
        leave();
        return false;
    }
    [[maybe_unused]] const uint64_t tp4 = FP_NOW();
    // ---- the true token bitmap: in a segment on the chain the marks before its first true
    // token are speculative (cleared), a segment off the chain is cleared whole; the chain's
    // walks past their segments (walk 2) then mark the tokens they passed
    const uint32_t vf = svfrom[g];
    const bool valid = vf != kMBad;
    {
        const uint32_t c1 = valid ? vf : s1;  // clear [s0, c1)
        for (uint32_t q = s0; q < c1;) {
            const uint32_t w = q >> 5, lo = q & 31u, hi = umin_(32u, c1 - (w << 5));
            const uint32_t mk = (hi == 32u ? ~0u : (1u << hi) - 1u) & (~0u << lo);
            atomicAnd(&bits[w], ~mk);
            q = (w + 1) << 5;
        }
    }
    __syncthreads();
    // ---- the chain's tokens past my segment (walk 2's positions, from my walk 1's exit to the
    // merge point) are true tokens too: mark them
    if (valid) {
        for (uint32_t q = x; q < C && q != m;) {
            atomicOr(&bits[q >> 5], 1u << (q & 31u));
            q = S3HC_HOPF(stage, mis, q, C).nxt;
        }
    }
    __syncthreads();
    [[maybe_unused]] const uint64_t tp5 = FP_NOW();
    // ---- sequence records, in stream order, and the lz4_flex bounds (every offset non-zero and
    // within the bytes produced before its match; output within the block limit and the caller's
    // capacity). Record: {lit | ll << 15, off | (ml - 4) << 16}, off = 0 for the last sequence
    // (no match).
    const uint32_t nbw = (C + 31u) / 32u;
    uint32_t wv[4], cnt = 0;
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
        const uint32_t k = 4u * g + j;
        wv[j] = k < nbw ? bits[k] : 0u;
        cnt += (uint32_t)__builtin_popcount(wv[j]);
    }
    uint32_t N;
    const uint32_t r0 = wg_excl_scan<TT / 64>(cnt, scr, &N);
    uint2* rec = a.rec + B.tok;
    uint32_t o = 0;
    int32_t minsl = 0x7FFFFFFF;
    bool bad = false;
    auto emitT = [&](uint32_t q, uint32_t k, const Tok& T) {  // the token at q (parsed: T) is sequence k
        const uint32_t lit = T.ll == 0 ? 0u : q + 1u + (T.ll >= 15u ? (T.ll - 15u) / 255u + 1u : 0u);
        o += T.ll;
        uint32_t y = 0;
        if (T.nxt != END) {
            bad |= T.off == 0u;
            minsl = min(minsl, (int32_t)o - (int32_t)T.off);
            o += T.ml;
            y = T.off | ((T.ml - 4u) << 16);
        }
#if S3HC_DTOK_SKIP & 1  // diagnostic builds: no record stores
        if (y == 0xFFFFFFFFu) rec[k] = make_uint2(lit | (T.ll << 15), y);
#else
        rec[k] = make_uint2(lit | (T.ll << 15), y);
#endif
    };
    auto emit = [&](uint32_t q, uint32_t k) {  // the token at q is sequence k
#if S3HC_DTOK_SKIP & 2  // diagnostic builds (timing only, output wrong): no token parse in the record pass
        Tok T;
        T.ll = q & 7u;
        T.ml = 4u + (q & 3u);
        T.off = 1u + (q & 15u);
        T.nxt = k + 1u == N ? END : q + 1u;
#else
        const Tok T = S3HC_HOPF(stage, mis, q, C);
#endif
        emitT(q, k, T);
    };
#if S3HC_DTOK_BAL == 1
    // balanced: thread g decodes sequences [g K, g K + K) (K = ceil(N / TT)), found from the
    // scanned per-thread counts (J[0] is free after the doubling) by binary search, then by the
    // bitmap words from there
    uint16_t* base = J[0];
    base[g] = (uint16_t)r0;
    if (g == 0) base[TT] = (uint16_t)N;
    __syncthreads();
    {
        const uint32_t K = (N + TT - 1u) / TT, R0 = g * K, R1 = umin_(N, R0 + K);
        if (R0 < R1) {
            uint32_t t = 0;
#pragma unroll
            for (uint32_t step = TT / 2; step; step >>= 1)
                if (base[t + step] <= R0) t += step;
            uint32_t w = 4u * t, xb = bits[w], skip = R0 - base[t];
            for (uint32_t pc = (uint32_t)__builtin_popcount(xb); skip >= pc; pc = (uint32_t)__builtin_popcount(xb)) {
                skip -= pc;
                xb = bits[++w];
            }
            for (; skip; --skip) xb &= xb - 1u;
            for (uint32_t k = R0; k < R1; ++k) {
                while (!xb) xb = bits[++w];
                const uint32_t q = (w << 5) + (uint32_t)__builtin_ctz(xb);
                xb &= xb - 1u;
                emit(q, k);
            }
        }
    }
#else
    // each thread decodes the true tokens of its four bitmap words (positions [128 g, 128 g + 128))
    // at its scanned rank
    uint32_t r = r0;
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
        uint32_t xb = wv[j];
        const uint32_t wb = (4u * g + j) << 5;
        while (xb) {
            const uint32_t q = wb + (uint32_t)__builtin_ctz(xb);
            xb &= xb - 1u;
            emit(q, r++);
        }
    }
#endif
    [[maybe_unused]] const uint64_t tp6 = FP_NOW();
    uint32_t Utot;
    const uint32_t obase = wg_excl_scan<TT / 64>(o, scr, &Utot);
    const bool fail = bad || (int64_t)obase + minsl < 0;
    if (fail) sflag[1] = 1u;
    __syncthreads();
    const bool ok = !sflag[1] && Utot <= B.limit && Utot <= B.cap;
    FastUnit F;
    F.ntok = N;
    F.U = Utot;
    F.pad0 = F.pad1 = 0;
    *fo = F;
    if (ok && !S3HC_DTOK_SKIP) {
        if (g == 0) {
            a.fu[u] = F;
            a.unit_fast[u] = 1;
        }
    } else {
        leave();  // (diagnostic skip builds: records are wrong, the per-unit decoder takes every block)
    }
#ifdef FPROF
    if ((g & 63u) == 0) {
        FP_ADD(0, tp1 - tp0);
        FP_ADD(1, tp2 - tp1);
        FP_ADD(2, tp3 - tp2);
        FP_ADD(3, tp4 - tp3);
        FP_ADD(4, tp5 - tp4);
        FP_ADD(5, tp6 - tp5);
        FP_ADD(6, FP_NOW() - tp0);
        FP_ADD(7, 1);
    }
#endif
    return ok;
}

// (unit_count: units [0, count) of a plan, from s3hc_kernels.hip, which this file is compiled inside)

__global__ __launch_bounds__(fst::kTT) void k_dtok(const uint8_t* __restrict__ src, const DecBlock* __restrict__ blk,
                                                   const DecUnit* __restrict__ units, uint32_t nunits,
                                                   const uint64_t* __restrict__ ucount,
                                                   const uint8_t* __restrict__ unit_lb, FastArgs a, uint32_t maxc) {
    const uint32_t nu = unit_count(ucount, nunits);
    for (uint32_t u = blockIdx.x; u < nu; u += gridDim.x) {
        FastUnit F;
        (void)dtok_unit<fst::kTT>(u, src, blk, units, unit_lb, a, maxc, &F);
        __syncthreads();  // (the next unit reuses the LDS)
    }
}

// ------------------------------------------------------------------ k_dexec
// One wave per block. Windows of 64 tokens (one sequence per lane; token positions from k_dtok,
// the token bytes and literals read straight from the compressed block in HBM/L2), executed in
// batches of <= kWin output bytes into an LDS ring of the block's recent output:
//   literals   every lane copies its literal run (16 bytes per step);
//   matches    sources older than the ring come from the block's output in HBM (flushed windows
//              ago), sources before the batch from the ring; sources inside the batch wait for
//              the first unfinished sequence: each round, the lowest lane still pending and every
//              pending lane whose source ends before that lane's match start copy (multi-round
//              resolution; log text needs ~5 rounds per 64 sequences);
//   flush      whole 1 KiB pieces of the ring to HBM.
// A sequence longer than kWin runs alone, wave-wide, in 1 KiB pieces (overlapping matches by
// growing multiples of their period).
#ifndef S3HC_DEX_PRIO  // 1: k_dexec's issue priority falls with its progress through the block
#define S3HC_DEX_PRIO 1
#endif
#ifndef S3HC_FXOR  // 1: a window's output range is cleared, then or-written (0: masked writes)
#define S3HC_FXOR 0
#endif
#ifndef S3HC_LIT32  // 1: the first literal chunk as four unaligned dword stores (0: 16 byte stores)
#define S3HC_LIT32 0
#endif
#ifndef S3HC_FXSKIP  // diagnostic builds: phases of k_dexec left out (timing only; output wrong)
#define S3HC_FXSKIP 0
#endif
namespace fst {
constexpr uint32_t kOR = 8192;       // output ring (bytes)
constexpr uint32_t kORW = kOR / 4;
constexpr uint32_t kORM = kOR - 1;
constexpr uint32_t kWin = 2048;      // output bytes of one batch, at most
constexpr uint32_t kFl = 1024;       // flush granule
constexpr uint32_t kGD = 4;          // pending-match dwords per lane held in registers
constexpr uint32_t kGW = 64 * kGD;
#ifndef S3HC_REDIR  // levels of sequence-level source redirection per window (0: off; round 6 A/B:
#define S3HC_REDIR 1  // one level 0.497 ms decode, none 0.518, two 0.510, three 0.551)
#endif
constexpr uint32_t kRedir = S3HC_REDIR;
static_assert(2 * kWin + kFl <= kOR, "far sources of a batch must be flushed before it runs");
}  // namespace fst

namespace {
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint4 uint4u __attribute__((aligned(1)));
typedef uint32_t u32u __attribute__((aligned(1)));

// 16 bytes at any global address (hardware unaligned access)
__device__ __forceinline__ uint4 gld16(const uint8_t* p) { return *(const uint4u*)p; }
__device__ __forceinline__ uint32_t gld4(const uint8_t* p) { return *(const u32u*)p; }

// 16 bytes at block byte p of a compressed block of C bytes: a block is always followed by at
// least 4 bytes of its frame (next block word or EndMark), so loads ending by C + 4 stay inside
// the frame; a load reaching further (the block's last literals) is done bytewise, zero-filled
__device__ __forceinline__ uint4 gld16_blk(const uint8_t* in, uint32_t p, uint32_t C) {
    if (p + 16u <= C + 4u) return gld16(in + p);
    uint32_t w[4] = {0u, 0u, 0u, 0u};
    for (uint32_t k = 0; k < 16u && p + k < C; ++k) w[k >> 2] |= (uint32_t)in[p + k] << (8u * (k & 3u));
    return make_uint4(w[0], w[1], w[2], w[3]);
}

// 16 bytes of the ring at byte position y (any alignment, wraps)
__device__ __forceinline__ uint4 rld16(const uint32_t* ring, uint32_t y) {
    const uint32_t A = y & fst::kORM, dw = A >> 2, sh = A & 3u;
    const uint32_t r0 = ring[dw], r1 = ring[(dw + 1) & (fst::kORW - 1)], r2 = ring[(dw + 2) & (fst::kORW - 1)];
    const uint32_t r3 = ring[(dw + 3) & (fst::kORW - 1)], r4 = ring[(dw + 4) & (fst::kORW - 1)];
    return make_uint4(__builtin_amdgcn_alignbyte(r1, r0, sh), __builtin_amdgcn_alignbyte(r2, r1, sh),
                      __builtin_amdgcn_alignbyte(r3, r2, sh), __builtin_amdgcn_alignbyte(r4, r3, sh));
}

typedef __attribute__((address_space(3))) uint32_t lds_u32;
__device__ __forceinline__ void mskor(uint32_t* lds_dw, uint32_t mask, uint32_t data) {
    const uint32_t addr = (uint32_t)(uintptr_t)(lds_u32*)lds_dw;  // LDS byte address
    asm volatile("ds_mskor_b32 %0, %1, %2" ::"v"(addr), "v"(mask), "v"(data & mask) : "memory");
}

// the first n (<= 16) bytes of v to the ring at byte position y, exactly (other lanes may be
// writing the neighbouring bytes of the first and last dword: masked atomic or-writes)
__device__ __forceinline__ void rst(uint32_t* ring, uint32_t y, uint4 v, uint32_t n) {
    if (n == 0) return;
    const uint32_t a = y & 3u, db = (y & fst::kORM) >> 2;
    const uint32_t s = 32u - 8u * a;  // v shifted up by a bytes: dword i = ({v_i, v_(i-1)} >> s)
    const uint32_t o0 = (uint32_t)(((uint64_t)v.x << 32) >> s);
    const uint32_t o1 = (uint32_t)((((uint64_t)v.y << 32) | v.x) >> s);
    const uint32_t o2 = (uint32_t)((((uint64_t)v.z << 32) | v.y) >> s);
    const uint32_t o3 = (uint32_t)((((uint64_t)v.w << 32) | v.z) >> s);
    const uint32_t o4 = (uint32_t)((uint64_t)v.w >> s);
    const uint32_t e = a + n;  // end byte in the 5-dword window (1..19)
    auto tmask = [](int x) -> uint32_t {  // bytes below x (clamped to 0..4)
        const uint32_t c = (uint32_t)min(max(x, 0), 4);
        return ~(uint32_t)(0xFFFFFFFFull << (8u * c));
    };
    const uint32_t m0 = tmask((int)e) & (0xFFFFFFFFu << (8u * a));
    const uint32_t m1 = tmask((int)e - 4), m2 = tmask((int)e - 8), m3 = tmask((int)e - 12), m4 = tmask((int)e - 16);
    mskor(ring + db, m0, o0);
    if (m1) mskor(ring + ((db + 1) & (fst::kORW - 1)), m1, o1);
    if (m2) mskor(ring + ((db + 2) & (fst::kORW - 1)), m2, o2);
    if (m3) mskor(ring + ((db + 3) & (fst::kORW - 1)), m3, o3);
    if (m4) mskor(ring + ((db + 4) & (fst::kORW - 1)), m4, o4);
}

// the same into ring bytes known to be zero (the window's output range is cleared before it
// runs): plain or-writes, no per-dword masks. v's bytes at and after n are dropped first; the
// five output dwords come from byte permutes of neighbouring source dwords.
__device__ __forceinline__ uint32_t keep_below(int x) {  // bytes below x (clamped to 0..4)
    const uint32_t c = (uint32_t)min(max(x, 0), 4);
    return ~(uint32_t)(0xFFFFFFFFull << (8u * c));
}
__device__ __forceinline__ void ds_or(uint32_t* lds_dw, uint32_t data) {
    __hip_atomic_fetch_or(lds_dw, data, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}
__device__ __forceinline__ void rst_or(uint32_t* ring, uint32_t y, uint4 v, uint32_t n) {
    const int ni = (int)n;
    v.x &= keep_below(ni);
    v.y &= keep_below(ni - 4);
    v.z &= keep_below(ni - 8);
    v.w &= keep_below(ni - 12);
    const uint32_t a = y & 3u, db = (y & fst::kORM) >> 2;
    // output byte j of dword i = source byte 4i + j - a: selector byte (j + 4 - a) picks from
    // {hi = v_i, lo = v_(i-1)}
    const uint32_t sel = 0x03020100u + (4u - a) * 0x01010101u;
    const uint32_t o0 = __builtin_amdgcn_perm(v.x, 0u, sel), o1 = __builtin_amdgcn_perm(v.y, v.x, sel);
    const uint32_t o2 = __builtin_amdgcn_perm(v.z, v.y, sel), o3 = __builtin_amdgcn_perm(v.w, v.z, sel);
    const uint32_t o4 = __builtin_amdgcn_perm(0u, v.w, sel);
    if (db + 4u < fst::kORW) {
        ds_or(ring + db, o0);
        ds_or(ring + db + 1, o1);
        ds_or(ring + db + 2, o2);
        ds_or(ring + db + 3, o3);
        if (o4) ds_or(ring + db + 4, o4);
    } else {
        ds_or(ring + db, o0);
        ds_or(ring + ((db + 1) & (fst::kORW - 1)), o1);
        ds_or(ring + ((db + 2) & (fst::kORW - 1)), o2);
        ds_or(ring + ((db + 3) & (fst::kORW - 1)), o3);
        if (o4) ds_or(ring + ((db + 4) & (fst::kORW - 1)), o4);
    }
}

// ring [from, from + n) -> 0 (wave-wide; n <= kOR): aligned 16-byte pieces plus masked edges
__device__ __forceinline__ void ring_clear(uint32_t* ring, uint32_t from, uint32_t n, uint32_t lane) {
    if (n == 0) return;
    const uint32_t to = from + n;
    const uint32_t a16 = (from + 15u) & ~15u, b16 = to & ~15u;
    if (a16 < b16) {
        for (uint32_t q = a16 + 16u * lane; q < b16; q += 1024u)
            *(uint4*)((uint8_t*)ring + (q & fst::kORM)) = make_uint4(0, 0, 0, 0);
    }
    // edges: the dwords of [from, min(a16, to)) and [max(b16, a16), to), lanes 0..3 and 4..7
    const uint32_t e0 = umin_(a16, to), s1 = umax_(b16, e0);
    const uint32_t d = lane < 4u ? (from & ~3u) + 4u * lane : s1 + 4u * (lane - 4u);
    const uint32_t lo = lane < 4u ? umax_(d, from) : d, hi = umin_(d + 4u, lane < 4u ? e0 : to);
    if (lane < 8u && lo < hi) {
        const uint32_t m = (0xFFFFFFFFu << (8u * (lo - d))) & keep_below((int)(hi - d));
        uint32_t* p = ring + ((d & fst::kORM) >> 2);
        if (m == 0xFFFFFFFFu) *p = 0u;
        else mskor(p, m, 0u);
    }
}

__device__ __forceinline__ void wr16(uint32_t* ring, uint32_t y, uint4 v, uint32_t n) {
#if S3HC_FXOR
    rst_or(ring, y, v, n);
#else
    rst(ring, y, v, n);
#endif
}

// ring [from, from + n) -> out + from, n <= kFl, the range contiguous in the ring
__device__ __forceinline__ void flush_piece(const uint32_t* ring, uint8_t* out, uint32_t from, uint32_t n, uint32_t lane) {
    const uint8_t* rb = (const uint8_t*)ring;
    if (n == fst::kFl) {
        const uint4 v = *(const uint4*)(rb + (from & fst::kORM) + 16u * lane);
        *(uint4u*)(out + from + 16u * lane) = v;
    } else {
        for (uint32_t k = lane; k < n; k += 64) out[from + k] = rb[(from + k) & fst::kORM];
    }
}
}  // namespace

namespace {
// Token decode of one window lane from its token dword w0 (token + 3 bytes at the token) and the
// dword w1 at the offset (offset + 2 bytes); runs of three or more extension bytes (rare) are
// read byte by byte. k_dtok validated the chain: every field is in bounds.
struct SeqF {
    uint32_t ll, lit, off, ml;
};
__device__ __forceinline__ uint32_t lit_len(const uint8_t* in, uint32_t pos, uint32_t w0, uint32_t& lit) {
    const uint32_t t = w0 & 0xFFu;
    uint32_t L = t >> 4, q = pos + 1;
    if (L == 15u) {
        uint32_t e = (w0 >> 8) & 0xFFu;
        L += e;
        ++q;
        if (e == 255u) {
            e = (w0 >> 16) & 0xFFu;
            L += e;
            ++q;
            while (e == 255u) {
                e = in[q++];
                L += e;
            }
        }
    }
    lit = q;
    return L;
}
__device__ __forceinline__ uint32_t match_len(const uint8_t* in, uint32_t mp, uint32_t t, uint32_t w1) {
    uint32_t M = (t & 15u) + 4u;
    if ((t & 15u) == 15u) {
        uint32_t f = (w1 >> 16) & 0xFFu;
        M += f;
        if (f == 255u) {
            f = w1 >> 24;
            M += f;
            uint32_t q2 = mp + 4;
            while (f == 255u) {
                f = in[q2++];
                M += f;
            }
        }
    }
    return M;
}
// DPP lane moves (row_shr / row_bcast; lanes without a source read 0) and wave-wide inclusive
// scans on them (no LDS round trip)
template <int CTRL, int ROWMASK>
__device__ __forceinline__ uint32_t fdpp(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROWMASK, 0xF, false);
}
__device__ __forceinline__ uint32_t incl_scan(uint32_t x, uint32_t) {
    x += fdpp<0x111, 0xF>(x);
    x += fdpp<0x112, 0xF>(x);
    x += fdpp<0x114, 0xF>(x);
    x += fdpp<0x118, 0xF>(x);
    x += fdpp<0x142, 0xA>(x);
    x += fdpp<0x143, 0xC>(x);
    return x;
}
__device__ __forceinline__ void wsync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// v shifted down by sh bytes (0..15), zeros shifted in
__device__ __forceinline__ uint4 shr16(uint4 v, uint32_t sh) {
    uint32_t w[8] = {v.x, v.y, v.z, v.w, 0u, 0u, 0u, 0u};
    const uint32_t k = sh >> 2, r = sh & 3u;
    uint32_t o[4];
#pragma unroll
    for (uint32_t i = 0; i < 4; ++i) {
        uint32_t lo = 0, hi = 0;
#pragma unroll
        for (uint32_t t = 0; t < 4; ++t) {
            lo = k == t ? w[i + t] : lo;
            hi = k == t ? w[i + t + 1] : hi;
        }
        o[i] = __builtin_amdgcn_alignbyte(hi, lo, r);
    }
    return make_uint4(o[0], o[1], o[2], o[3]);
}
__device__ __forceinline__ uint32_t incl_max(uint32_t x) {
    x = umax_(x, fdpp<0x111, 0xF>(x));
    x = umax_(x, fdpp<0x112, 0xF>(x));
    x = umax_(x, fdpp<0x114, 0xF>(x));
    x = umax_(x, fdpp<0x118, 0xF>(x));
    x = umax_(x, fdpp<0x142, 0xA>(x));
    x = umax_(x, fdpp<0x143, 0xC>(x));
    return x;
}
}  // namespace

// lane l's value of x (l wave-uniform): v_readlane, no LDS round trip (unlike __shfl's ds_bpermute)
__device__ __forceinline__ uint32_t rdlane(uint32_t x, uint32_t l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)x, (int)l);
}

// An executor wave's LDS besides its ring (k_dexec runs four executors per workgroup)
struct DexLds {
    uint4 pinfo[64];
    uint8_t gmk[fst::kGW];
    uint32_t segs[64];  // redirection: each lane's sequence end (window offset, inclusive scan)
    uint32_t samp[8];   // segs[8k + 7]: the first level of the owner search
};

// One wave executes unit u (taken by the token index: F = its sequences and bytes) into the
// 8 KiB LDS ring `ring`. hsync (k_dsmall, nullptr otherwise): a hashing wave of the workgroup
// reads the ring behind the executor; hsync[0] = bytes final (published after each window),
// hsync[1] = bytes hashed; the executor never overwrites ring bytes that are not hashed yet.
__device__ __forceinline__ void dexec_unit(const uint32_t u, const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                           const DecBlock* __restrict__ blk, const DecUnit* __restrict__ units,
                                           uint32_t* __restrict__ blk_out, int32_t* __restrict__ blk_status,
                                           const FastArgs& a, const FastUnit F, uint32_t* __restrict__ ring,
                                           volatile uint32_t* hsync, DexLds* __restrict__ dl) {
    using namespace fst;
    uint4* pinfo = dl->pinfo;  // pending matches: md, ms, ml | off << 16, first dword - rank
    uint8_t* gmk = dl->gmk;    // pending dwords: rank of each lane's first dword -> lane + 1
    const uint32_t lane = threadIdx.x & 63u;
    const DecUnit Un = units[u];
    const DecBlock B = blk[Un.first];
    // ring bytes [end - kOR + 16, end) may be overwritten once the hashing wave is past them;
    // bytes below upos are published to it after every window / batch / piece
    auto hwait = [&](uint32_t end) {
        if (hsync)
            while (end + 16u > hsync[1] + kOR) __builtin_amdgcn_s_sleep(1);
    };
    auto hpub = [&](uint32_t done) {
        if (hsync) {
            // the ring bytes before the progress word (LDS only: a workgroup-scope fence would
            // also drain this wave's global prefetches)
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (lane == 0) hsync[0] = done;
        }
    };
    const uint8_t* in = src + B.src_off;
    uint8_t* out = dst + B.dst_off;
    const uint2* rec = a.rec + B.tok;
    const uint32_t N = F.ntok, C = B.csize;
    uint32_t upos = 0, flushed = 0;
    auto flush_full = [&]() {
        while (upos - flushed >= kFl) {
            if (!(S3HC_FXSKIP & 16)) flush_piece(ring, out, flushed, kFl, lane);
            flushed += kFl;
        }
    };
    const uint32_t nwin = (N + 63u) >> 6;
    // my sequence record in window w (zeros past the last: no literal, no match); the load is
    // unconditional (a clamped index), so no branch forces an early wait
    auto ldrec = [&](uint32_t w) -> uint2 {
        const uint32_t t = 64u * w + lane;
        const uint2 v = rec[t < N ? t : N - 1u];
        return t < N ? v : make_uint2(0u, 0u);
    };
    auto unpack = [&](uint2 r) -> SeqF {
        SeqF f;
        f.ll = r.x >> 15;
        f.lit = f.ll ? (r.x & 0x7FFFu) : C;
        f.off = r.y & 0xFFFFu;
        f.ml = f.off ? (r.y >> 16) + 4u : 0u;
        return f;
    };
    // ---- pipeline prologue: records of windows 1 and 2 in flight, window 0 unpacked
    uint2 r_n = ldrec(1), r_2 = ldrec(2);
    SeqF fc = unpack(ldrec(0)), fn;
    uint32_t Sincl_c = incl_scan(fc.ll + fc.ml, lane);
    uint32_t S_c = rdlane(Sincl_c, 63);
    bool far_c = false, pf_c = S_c <= kWin;  // window 0: nothing is far
    uint4 lit0_c, lit1_c, far0_c = make_uint4(0, 0, 0, 0), far1_c = far0_c;
    uint32_t lsh_c;
    {
        const int32_t lim = (int32_t)C + 4 - 16;
        const uint32_t lit = fc.ll ? fc.lit : C;
        const int32_t q0 = min((int32_t)lit, max(lim, -11)), q1 = min((int32_t)lit + 16, max(lim, -11));
        lit0_c = gld16(in + q0);
        lit1_c = gld16(in + q1);
        lsh_c = (lit - (uint32_t)q0) | ((lit + 16u - (uint32_t)q1) << 8);
    }
    [[maybe_unused]] const uint64_t te0 = FP_NOW();
#ifdef UPROF
    const uint64_t tr0 = __builtin_amdgcn_s_memrealtime();  // (constant 100 MHz clock, chip-wide)
#endif
    [[maybe_unused]] uint64_t tsum[6] = {0, 0, 0, 0, 0, 0};
    uint32_t nrounds = 0;
    for (uint32_t w = 0; w < nwin; ++w) {
        [[maybe_unused]] uint64_t tq0 = FP_NOW();
#if S3HC_DEX_PRIO
        // issue priority falls with progress (3 in the first quarter of the block's windows, 0 in
        // the last): the SIMD's arbiter otherwise favours its oldest wave, so the executors of a
        // one-pass batch finish one after another and the last runs alone, its latency unhidden
        {
            const uint32_t pq = umin_(3u, (4u * w) / nwin);  // (wave-uniform; the priority is an immediate)
            if (pq == 0) __builtin_amdgcn_s_setprio(3);
            else if (pq == 1) __builtin_amdgcn_s_setprio(2);
            else if (pq == 2) __builtin_amdgcn_s_setprio(1);
            else __builtin_amdgcn_s_setprio(0);
        }
#endif
        const uint32_t nact = umin_(64u, N - 64u * w);
        const bool act = lane < nact;
        // ---- stage A: window w+3's records (two windows of lead); stage C: window w+1 unpacked,
        // its literals and far match sources prefetched
        const uint2 r_3 = ldrec(w + 3);
        fn = unpack(r_n);
        const uint32_t Sincl_n = incl_scan(fn.ll + fn.ml, lane);
        const uint32_t S_n = rdlane(Sincl_n, 63);
        const bool pf_n = S_c <= kWin && S_n <= kWin;
        // literal chunks at clamped in-frame addresses (a frame holds >= 11 bytes before a block's
        // payload and >= 4 after it); the shift back to the literal start is applied at use
        const int32_t lim = (int32_t)C + 4 - 16;
        const int32_t q0 = min((int32_t)fn.lit, max(lim, -11)), q1 = min((int32_t)fn.lit + 16, max(lim, -11));
        const uint4 lit0_n = gld16(in + q0), lit1_n = gld16(in + q1);
        const uint32_t lsh_n = (fn.lit - (uint32_t)q0) | ((fn.lit + 16u - (uint32_t)q1) << 8);
        bool far_n = false;
        const uint8_t* fa0 = in - 11;
        if (pf_n && fn.ml) {
            const uint32_t upos_n = upos + S_c;
            const uint32_t md = upos_n + Sincl_n - fn.ml, ms = md - fn.off;
            far_n = ms + kOR < upos_n + S_n && ms < md;
            if (far_n) fa0 = out + ms;
        }
        const uint4 far0_n = gld16(fa0), far1_n = gld16(far_n ? fa0 + 16 : fa0);
#ifdef FPROF
        { const uint64_t tn = FP_NOW(); tsum[0] += tn - tq0; tq0 = tn; }
#endif
        // ---- execute window w
        const uint32_t ll = act ? fc.ll : 0u, lit = fc.lit, off = fc.off, ml = act ? fc.ml : 0u;
        const uint32_t len = ll + ml;
        if (pf_c && S_c <= kWin) {
            hwait(upos + S_c);
            const uint32_t d0 = upos + Sincl_c - len;
            // literals (first 32 bytes prefetched; near the block's end they were loaded from a
            // clamped address: shift them back)
            if (__ballot(act && ll && (lsh_c & 0xFFFFu))) {
                if (lsh_c & 0xFFu) lit0_c = shr16(lit0_c, lsh_c & 0xFFu);
                if (lsh_c & 0xFF00u) lit1_c = shr16(lit1_c, (lsh_c >> 8) & 0xFFu);
            }
            if (S3HC_FXOR && !(S3HC_FXSKIP & 8)) ring_clear(ring, upos, S_c, lane);
            wsync();
            if (!(S3HC_FXSKIP & 2) && __ballot(act && ll > 16u)) {
                // second chunk first (same rule as the first chunk below: its bytes past the
                // run land in this lane's match or in later lanes' bytes, stored after them)
                const uint32_t A1 = (d0 + 16u) & kORM;
                const bool bytew2 = !S3HC_FXOR && act && ll > 16u && A1 + 16u <= kOR && d0 + 32u <= upos + S_c;
                if (bytew2) {
                    uint8_t* rb = (uint8_t*)ring + A1;
                    const uint32_t x[4] = {lit1_c.x, lit1_c.y, lit1_c.z, lit1_c.w};
#pragma unroll
                    for (int k = 15; k >= 0; --k) {
                        rb[k] = (uint8_t)(x[k >> 2] >> (8 * (k & 3)));
                        __builtin_amdgcn_sched_barrier(0);  // (the stores' order is the contract)
                    }
                }
                asm volatile("" ::: "memory");
                if (act && ll > 16u && !bytew2) wr16(ring, d0 + 16u, lit1_c, umin_(16u, ll - 16u));
            }
            if (!(S3HC_FXSKIP & 2)) {
                // first literal chunk as 16 plain byte stores, last byte first: bytes past a
                // lane's literals land in its own match or in later lanes' bytes, which are
                // all stored after them (later lanes' first chunks by a later store of this
                // sequence; matches and further chunks after it); lanes whose chunk would wrap
                // the ring or pass the window's end take the masked write
                const uint32_t A0 = d0 & kORM;
                const bool bytew = !S3HC_FXOR && act && ll && A0 + 16u <= kOR && d0 + 16u <= upos + S_c;
                if (bytew) {
                    uint8_t* rb = (uint8_t*)ring + A0;
#if S3HC_LIT32
                    // four unaligned dword stores, highest first: a lane's bytes past its
                    // literals that land in a later lane's literals sit >= 5 bytes further into
                    // this lane's chunk (ll >= 1, ml >= 4), so always in a higher dword, stored
                    // by an earlier instruction than the later lane's own store of that byte
                    *(u32u*)(rb + 12) = lit0_c.w;
                    __builtin_amdgcn_sched_barrier(0);
                    *(u32u*)(rb + 8) = lit0_c.z;
                    __builtin_amdgcn_sched_barrier(0);
                    *(u32u*)(rb + 4) = lit0_c.y;
                    __builtin_amdgcn_sched_barrier(0);
                    *(u32u*)(rb + 0) = lit0_c.x;
                    __builtin_amdgcn_sched_barrier(0);
#else
                    const uint32_t x[4] = {lit0_c.x, lit0_c.y, lit0_c.z, lit0_c.w};
#pragma unroll
                    for (int k = 15; k >= 0; --k) {
                        rb[k] = (uint8_t)(x[k >> 2] >> (8 * (k & 3)));
                        __builtin_amdgcn_sched_barrier(0);  // (the stores' order is the contract)
                    }
#endif
                }
                asm volatile("" ::: "memory");
                if (act && ll && !bytew) wr16(ring, d0, lit0_c, umin_(16u, ll));
            }
            for (uint32_t c = 32; __ballot(act && c < ll); c += 16u)
                if (act && c < ll) wr16(ring, d0 + c, gld16_blk(in, lit + c, C), umin_(16u, ll - c));
#ifdef FPROF
            __builtin_amdgcn_s_waitcnt(0);
            { const uint64_t tn = FP_NOW(); tsum[1] += tn - tq0; tq0 = tn; }
#endif
            const uint32_t md = d0 + ll, ms = md - off;
            const bool hasm = act && ml > 0;
            const bool far = hasm && far_c;
            bool pend = hasm && !far && ms + ml > upos;
            // ---- sequence-level source redirection (round 6). A pending match whose source lies
            // inside the literals of one sequence of this window is final before round 0 (literals
            // are stored first); one whose source lies inside the match of one non-overlapping
            // sequence of the window copies from that sequence's source instead (the offset into
            // it carries over): when that source is final (not pending, or before the window) the
            // match becomes a round-0 item (16-byte copies, no dword sweeps), otherwise it keeps
            // the sweeps below with the redirected source (same bytes, a shorter chain). kRedir
            // levels repeat the step through pending owners; one level measured fastest (the
            // levels' LDS round trips cost more than the sweeps they save). Sources straddling
            // sequences, and overlapping copies, keep the sweeps.
            uint32_t src = ms;    // the match's source (redirected)
            bool rfar = false;    // a redirected source older than the ring: read from HBM
            if (kRedir && __ballot(pend && off >= ml && ms >= upos)) {
                bool cand = pend && off >= ml && ms >= upos;
                bool redir = false;
                dl->segs[lane] = Sincl_c;
                if ((lane & 7u) == 7u) dl->samp[lane >> 3] = Sincl_c;
                for (uint32_t lev = 0; lev < kRedir; ++lev) {
                    // snapshot of the window's sequences: match start, current source, (ml, ll),
                    // bit 0 = its current source holds final bytes before round 0 (not pending, or
                    // resolved at an earlier level), bit 1 = it does not overlap itself
                    pinfo[lane] = make_uint4(md, src, ml | (ll << 16),
                                             (pend && !redir ? 0u : 1u) | (off >= ml ? 2u : 0u));
                    wsync();
                    if (cand) {
                        // the sequence owning window offset r: the lanes whose end is <= r, counted
                        // over 8 samples, then over the 8 ends of that bucket (samp[7] = S_c > r)
                        const uint32_t r = src - upos;
                        const uint4 sa = *(const uint4*)&dl->samp[0], sb = *(const uint4*)&dl->samp[4];
                        const uint32_t b = (uint32_t)(sa.x <= r) + (uint32_t)(sa.y <= r) + (uint32_t)(sa.z <= r) +
                                           (uint32_t)(sa.w <= r) + (uint32_t)(sb.x <= r) + (uint32_t)(sb.y <= r) +
                                           (uint32_t)(sb.z <= r);
                        const uint4 ta = *(const uint4*)&dl->segs[8u * b], tb = *(const uint4*)&dl->segs[8u * b + 4u];
                        const uint32_t j = 8u * b + (uint32_t)(ta.x <= r) + (uint32_t)(ta.y <= r) + (uint32_t)(ta.z <= r) +
                                           (uint32_t)(ta.w <= r) + (uint32_t)(tb.x <= r) + (uint32_t)(tb.y <= r) +
                                           (uint32_t)(tb.z <= r);
                        const uint4 Pj = pinfo[j];
                        const uint32_t mdj = Pj.x, mlj = Pj.z & 0xFFFFu, dj = mdj - (Pj.z >> 16);
                        if (src >= dj && src + ml <= mdj) {  // inside its literals
                            cand = false;
                            redir = true;
                        } else if (src >= mdj && src + ml <= mdj + mlj && (Pj.w & 2u)) {  // inside its match
                            // (the owner's source is final, or the new source lies wholly before
                            // the window: done; else look again while it lies in the window. A
                            // source left pending stays in the ring: a far owner source is final)
                            src = Pj.y + (src - mdj);
                            redir = (Pj.w & 1u) != 0u || src + ml <= upos;
                            cand = !redir && src >= upos;
                        } else {
                            cand = false;  // straddles sequences, or the owner overlaps itself
                        }
                    }
                    if (lev + 1u < kRedir) {
                        wsync();
                        if (!__ballot(cand)) break;
                    }
                }
                wsync();  // (round 0 rewrites pinfo)
                if (redir) {
                    pend = false;
                    rfar = src + kOR < upos + S_c;
                }
            }
            // round 0: far sources (prefetched) and sources before the window (an overlapping
            // match is always pending: its source reaches its own output)
            if (!(S3HC_FXSKIP & 4) && hasm && !pend) {
                if (far) {
                    wr16(ring, md, far0_c, umin_(16u, ml));
                    if (ml > 16u) wr16(ring, md + 16u, far1_c, umin_(16u, ml - 16u));
                }
            }
            // the rest of round 0 load-balanced over the lanes: every 16-byte chunk of every such
            // match (a far match's first 32 bytes came prefetched) is one work item, items are
            // dealt out 64 at a time (the owner of item j: start marks + max-scan); a window's
            // <= kWin bytes make <= 192 items
            {
                const uint32_t c0 = far ? 32u : 0u;
                const uint32_t nch = !(S3HC_FXSKIP & 4) && hasm && !pend && ml > c0 ? (ml - c0 + 15u) >> 4 : 0u;
                const uint32_t chincl = incl_scan(nch, lane);
                const uint32_t T0 = rdlane(chincl, 63);
                if (T0) {
                    pinfo[lane] = make_uint4(md + c0, src + c0, (ml - c0) | (far || rfar ? 0x10000u : 0u), chincl - nch);
                    ((uint32_t*)gmk)[lane] = 0u;
                    wsync();
                    if (nch) gmk[chincl - nch] = (uint8_t)(lane + 1u);
                    wsync();
                    uint32_t carry = 0;
                    for (uint32_t j0 = 0; j0 < T0; j0 += 64u) {
                        const uint32_t j = j0 + lane;
                        const uint32_t own = umax_(incl_max(j < T0 ? (uint32_t)gmk[j] : 0u), carry);
                        carry = rdlane(own, 63);
                        if (j < T0) {
                            const uint4 P = pinfo[own - 1u];
                            const uint32_t c = 16u * (j - P.w), rem = P.z & 0xFFFFu;
                            uint4 v;
                            if (P.z >> 16) v = gld16(out + P.y + c);
                            else v = rld16(ring, P.y + c);
                            wr16(ring, P.x + c, v, umin_(16u, rem - c));
                        }
                    }
                    wsync();
                }
            }
#ifdef FPROF
            __builtin_amdgcn_s_waitcnt(0);
            { const uint64_t tn = FP_NOW(); tsum[2] += tn - tq0; tq0 = tn; }
#endif
            // in-window sources: every output dword of a pending match is given to one lane
            // (packed over the lanes), and each such dword is re-gathered from its sources until a
            // whole sweep changes nothing: at that fixed point every byte equals its source, whose
            // chain ends in a final byte, so every byte is final (sweeps ~ chain depth + 1)
            if (!(S3HC_FXSKIP & 1) && __ballot(pend)) {
                const uint32_t df = md >> 2, cnt = pend ? ((md + ml - 1u) >> 2) - df + 1u : 0u;
                const uint32_t cincl = incl_scan(cnt, lane);
                const uint32_t T = rdlane(cincl, 63);
                if (T <= 64u * kGD) {
                    pinfo[lane] = make_uint4(md, src, ml | (off << 16), df - (cincl - cnt));
                    ((uint32_t*)gmk)[lane] = 0u;  // kGW = 256 mark bytes
                    wsync();
                    if (cnt) gmk[cincl - cnt] = (uint8_t)(lane + 1u);
                    wsync();
                    uint32_t gd[kGD], gm[kGD], ga[kGD], go[kGD];
                    uint32_t carry = 0;
#pragma unroll
                    for (uint32_t i = 0; i < kGD; ++i) {
                        if (64u * i >= T) break;
                        const uint32_t j = lane + 64u * i;
                        const uint32_t own = umax_(incl_max(j < T ? (uint32_t)gmk[j] : 0u), carry);
                        carry = rdlane(own, 63);
                        gd[i] = 0xFFFFFFFFu;
                        gm[i] = ga[i] = go[i] = 0;
                        if (j < T && own) {
                            const uint4 P = pinfo[own - 1u];
                            const uint32_t d = P.w + j, b0 = d << 2, pmd = P.x, pml = P.z & 0xFFFFu;
                            const uint32_t lo = pmd > b0 ? pmd - b0 : 0u, hi = umin_(4u, pmd + pml - b0);
                            gd[i] = d;
                            gm[i] = (hi >= 4u ? ~0u : (1u << (8u * hi)) - 1u) & (~0u << (8u * lo));
                            ga[i] = P.y + b0 - pmd;  // source of the dword's byte 0 (non-overlapping)
                            const uint32_t poff = P.z >> 16;
                            if (poff < pml) {
                                // overlapping: byte b copies the byte (b - md) mod off into the
                                // match's first period; the four ring indices, found once here
                                // (one division) instead of in every sweep
                                const int32_t e0 = (int32_t)b0 - (int32_t)pmd;
                                const uint32_t base = e0 > 0 ? (uint32_t)e0 : 0u;
                                const uint32_t rr = base % poff;
                                uint32_t sx[4];
#pragma unroll
                                for (uint32_t q = 0; q < 4u; ++q) {
                                    const int32_t e = e0 + (int32_t)q;
                                    uint32_t x = e > 0 ? rr + ((uint32_t)e - base) : 0u;
                                    x = poff == 1u ? 0u : x;
                                    x -= x >= poff ? poff : 0u;
                                    x -= x >= poff ? poff : 0u;
                                    sx[q] = (P.y + x) & kORM;
                                }
                                ga[i] = sx[0] | (sx[1] << 16);
                                go[i] = sx[2] | (sx[3] << 16) | 0x80000000u;  // (ring indices < 2^13)
                            }
                        }
                    }
                    // slot by slot: a slot's dwords only read lower addresses (earlier slots, already
                    // final, or lower dwords of the same slot), so each slot is swept to its own
                    // fixed point once the slots before it are final
#pragma unroll
                    for (uint32_t i = 0; i < kGD; ++i) {
                        if (64u * i >= T) break;
                        for (uint32_t sweeps = 0;; ++sweeps) {
                            bool chg = false;
                            if (gd[i] == 0xFFFFFFFFu) goto next_sweep;
                            {
                            uint32_t* rd = ring + (gd[i] & (kORW - 1));
                            const uint32_t cur = *rd;
                            uint32_t v;
                            if (!go[i]) {
                                const uint32_t A = ga[i];
                                v = __builtin_amdgcn_alignbyte(ring[((A >> 2) + 1u) & (kORW - 1)],
                                                               ring[(A >> 2) & (kORW - 1)], A & 3u);
                            } else {
                                const uint8_t* rb = (const uint8_t*)ring;
                                const uint32_t A = ga[i], Bq = go[i];
                                v = (uint32_t)rb[A & 0xFFFFu] | ((uint32_t)rb[A >> 16] << 8) |
                                    ((uint32_t)rb[Bq & 0x7FFFu] << 16) | ((uint32_t)rb[(Bq >> 16) & 0x7FFFu] << 24);
                            }
                            if (((cur ^ v) & gm[i]) != 0u) {
                                chg = true;
                                mskor(rd, gm[i], v);
                            }
                            }
                        next_sweep:
                            ++nrounds;
                            if (!__ballot(chg) || sweeps > 8192u) break;  // (a bound, never reached)
                        }
                    }
                } else {
                    // (more pending output than the registers hold: multi-round resolution, the
                    // lowest pending lane and every pending lane whose source ends before it)
                    for (;;) {
                        const uint64_t pm = __ballot(pend);
                        if (!pm) break;
                        const uint32_t first = (uint32_t)__builtin_ctzll(pm);
                        const uint32_t h = rdlane(md, (int)first);
                        const bool run = pend && (lane == first || (off >= ml && src + ml <= h));
                        const uint32_t step = off < 16u ? off : 16u;
                        for (uint32_t c = 0; __ballot(run && c < ml); c += step)
                            if (run && c < ml) rst(ring, md + c, rld16(ring, src + c), umin_(step, ml - c));
                        pend = pend && !run;
                        ++nrounds;
                    }
                }
            }
#ifdef FPROF
            __builtin_amdgcn_s_waitcnt(0);
            { const uint64_t tn = FP_NOW(); tsum[3] += tn - tq0; tq0 = tn; }
#endif
            upos += S_c;
            flush_full();
            hpub(upos);
        } else {
            // ---- a window of more than kWin output bytes (or right after one): batches of
            // <= kWin bytes in lane order, sources read at once; sequences longer than a batch run
            // alone, wave-wide
            uint32_t i0 = 0;
            while (i0 < nact) {
                const uint32_t base = i0 ? rdlane(Sincl_c, (int)(i0 - 1)) : 0u;
                const uint64_t fit = __ballot(act && lane >= i0 && Sincl_c - base <= kWin);
                const uint32_t i1 = fit ? 64u - (uint32_t)__builtin_clzll(fit) : i0;
                if (i1 <= i0) {
                    const uint32_t sll = rdlane(ll, (int)i0), slit = rdlane(lit, (int)i0);
                    const uint32_t soff = rdlane(off, (int)i0), sml = rdlane(ml, (int)i0);
                    for (uint32_t k = 0; k < sll; k += kFl) {
                        const uint32_t piece = umin_(kFl, sll - k);
                        const uint32_t j = 16u * lane;
                        hwait(upos + piece);
                        if (j < piece) rst(ring, upos + j, gld16_blk(in, slit + k + j, C), umin_(16u, piece - j));
                        upos += piece;
                        flush_full();
                        hpub(upos);
                    }
                    const uint32_t mdst = upos;
                    for (uint32_t k = 0; k < sml;) {
                        uint32_t piece = umin_(kFl, sml - k), P = soff;
                        if (soff < piece) {
                            P = soff * ((piece + soff - 1) / soff);
                            if (P > k + soff) P = soff * ((k + soff) / soff);
                            piece = umin_(piece, P);
                        }
                        hwait(upos + piece);
                        const uint32_t j = 16u * lane;
                        if (j < piece) {
                            const uint32_t y = mdst + k - P + j, n = umin_(16u, piece - j);
                            uint4 v;
                            if (y + kOR < upos + piece && y < upos) v = gld16(out + y);
                            else v = rld16(ring, y);
                            rst(ring, upos + j, v, n);
                        }
                        k += piece;
                        upos += piece;
                        flush_full();
                        hpub(upos);
                    }
                    i0 = i0 + 1;
                    continue;
                }
                const bool inb = act && lane >= i0 && lane < i1;
                const uint32_t Sb = rdlane(Sincl_c, (int)(i1 - 1)) - base;
                hwait(upos + Sb);
                const uint32_t d0 = upos + Sincl_c - len - base;
                for (uint32_t c = 0; __ballot(inb && c < ll); c += 16u)
                    if (inb && c < ll) rst(ring, d0 + c, gld16_blk(in, lit + c, C), umin_(16u, ll - c));
                const uint32_t md = d0 + ll, ms = md - off;
                const bool hasm = inb && ml > 0;
                const bool far = hasm && ms + kOR < upos + Sb && ms < md;
                bool pend = hasm && !far && ms + ml > upos;
                bool run = hasm && !pend;
                const uint32_t step = off < 16u ? off : 16u;
                for (;;) {
                    for (uint32_t c = 0; __ballot(run && c < ml); c += step) {
                        if (run && c < ml) {
                            uint4 v;
                            if (far) v = gld16(out + ms + c);
                            else v = rld16(ring, ms + c);
                            rst(ring, md + c, v, umin_(step, ml - c));
                        }
                    }
                    const uint64_t pm = __ballot(pend);
                    if (!pm) break;
                    const uint32_t first = (uint32_t)__builtin_ctzll(pm);
                    const uint32_t h = rdlane(md, (int)first);
                    run = pend && (lane == first || (off >= ml && ms + ml <= h));
                    pend = pend && !run;
                }
                upos += Sb;
                flush_full();
                hpub(upos);
                i0 = i1;
            }
        }
#ifdef FPROF
        __builtin_amdgcn_s_waitcnt(0);
        { const uint64_t tn = FP_NOW(); tsum[4] += tn - tq0; tq0 = tn; }
#endif
        // ---- rotate the pipeline
        fc = fn;
        Sincl_c = Sincl_n;
        S_c = S_n;
        pf_c = pf_n;
        far_c = far_n;
        lit0_c = lit0_n;
        lit1_c = lit1_n;
        lsh_c = lsh_n;
        far0_c = far0_n;
        far1_c = far1_n;
        r_n = r_2;
        r_2 = r_3;
    }
    hpub(upos);
    // ---- the rest of the output (< kFl bytes)
    if (upos > flushed) {
        const uint32_t n = upos - flushed, first = kOR - (flushed & kORM);
        if (n <= first) flush_piece(ring, out, flushed, n, lane);
        else {
            flush_piece(ring, out, flushed, first, lane);
            flush_piece(ring, out, flushed + first, n - first, lane);
        }
    }
    if (lane == 0) {
        blk_out[Un.first] = upos;
        blk_status[Un.first] = S3HC_OK;
    }
#ifdef FPROF
    if (lane == 0) {
        for (int k = 0; k < 5; ++k) FP_ADD(16 + k, tsum[k]);
        FP_ADD(21, FP_NOW() - te0);
        FP_ADD(22, nwin);
        FP_ADD(23, nrounds);
        FP_ADD(24, 1);
        // the spread of the units' lives (one pass holds the whole batch: the launch lasts as long
        // as its slowest wave): the longest, a histogram, the first start and the last end
        const uint64_t tend = FP_NOW(), tot = tend - te0;
        atomicMax(&g_fprof[31], (unsigned long long)tot);
        FP_ADD(tot < 600000u ? 12 : (tot < 900000u ? 13 : (tot < 1200000u ? 14 : 15)), 1);
        atomicMax(&g_fprof[8], (unsigned long long)~te0);
        atomicMax(&g_fprof[11], (unsigned long long)tend);
        atomicMax(&g_fprof[9], (unsigned long long)nwin);
    }
#endif
#ifdef UPROF
    if (lane == 0 && u < 8192u) {
        g_uprof[u][0] = tr0;
        g_uprof[u][1] = __builtin_amdgcn_s_memrealtime();
        g_uprof[u][2] = (unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 4);  // HW_ID
        g_uprof[u][3] = (unsigned long long)(__builtin_amdgcn_s_getreg((15 << 11) | 20) & 15u) |  // XCC_ID
                        ((unsigned long long)nrounds << 8) | ((unsigned long long)nwin << 32);
    }
#endif
}

#ifndef S3HC_SMALL_JUMP  // 1: small launches decode by pointer jumping (k_djump), 0: k_dsmall's executor
#define S3HC_SMALL_JUMP 1
#endif
// ------------------------------------------------------------------ k_dsmall
namespace {
constexpr uint32_t XH1 = 2654435761U, XH2 = 2246822519U, XH3 = 3266489917U, XH4 = 668265263U, XH5 = 374761393U;
__device__ __forceinline__ uint32_t xh_rotl(uint32_t x, int r) { return __builtin_amdgcn_alignbit(x, x, 32 - r); }
__device__ __forceinline__ uint32_t xh_round(uint32_t acc, uint32_t in) { return xh_rotl(acc + in * XH2, 13) * XH1; }
}  // namespace

// The hashing wave of k_dsmall: xxh32 (seed 0) of the unit's U output bytes, read from the
// executor's LDS ring behind it (hsync protocol of dexec_unit). Lane a = lane & 3 runs accumulator
// a; for 16 stripes at a time lane 4k + a loads stripe k's dword a and multiplies it by P2 (off the
// chain), the chain then adds, rotates and multiplies by P1 (k_lb_run's hashing wave, §4b).
__device__ __forceinline__ uint32_t hash_ring(const uint32_t* ring, volatile uint32_t* hsync, uint32_t U) {
    using namespace fst;
    const uint32_t lane = threadIdx.x & 63u, ha = lane & 3u;
    uint32_t hacc = ha == 0 ? XH1 + XH2 : (ha == 1 ? XH2 : (ha == 2 ? 0u : 0u - XH1));
    const uint32_t hns = U >> 4;
    uint32_t hs = 0;
    for (;;) {
        const uint32_t avail = hsync[0];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const uint32_t lim = umin_(avail >> 4, hns);
        for (; hs + 16u <= lim; hs += 16u) {
            const uint32_t mv = ring[((16u * hs + 4u * lane) & kORM) >> 2] * XH2;
            uint32_t m[16];
#pragma unroll
            for (uint32_t k = 0; k < 16; ++k) m[k] = (uint32_t)__shfl((int)mv, (int)(4u * k + ha), 64);
#pragma unroll
            for (uint32_t k = 0; k < 16; ++k) hacc = xh_rotl(hacc + m[k], 13) * XH1;
        }
        for (; hs < lim; ++hs) hacc = xh_round(hacc, ring[((16u * hs + 4u * ha) & kORM) >> 2]);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // (ring reads done before the slots are released)
        if (lane == 0) hsync[1] = 16u * hs;
        if (avail >= U) break;
        __builtin_amdgcn_s_sleep(2);
    }
    const int qb = (int)(lane & ~3u);
    const uint32_t v1 = (uint32_t)__shfl((int)hacc, qb, 64), v2 = (uint32_t)__shfl((int)hacc, qb + 1, 64);
    const uint32_t v3 = (uint32_t)__shfl((int)hacc, qb + 2, 64), v4 = (uint32_t)__shfl((int)hacc, qb + 3, 64);
    uint32_t h = U >= 16u ? xh_rotl(v1, 1) + xh_rotl(v2, 7) + xh_rotl(v3, 12) + xh_rotl(v4, 18) : XH5;
    h += U;
    const uint8_t* rb = (const uint8_t*)ring;
    uint32_t p = hns * 16u;
    for (; p + 4u <= U; p += 4u) {
        const uint32_t w = (uint32_t)rb[p & kORM] | ((uint32_t)rb[(p + 1u) & kORM] << 8) |
                           ((uint32_t)rb[(p + 2u) & kORM] << 16) | ((uint32_t)rb[(p + 3u) & kORM] << 24);
        h = xh_rotl(h + w * XH3, 17) * XH4;
    }
    for (; p < U; ++p) h = xh_rotl(h + (uint32_t)rb[p & kORM] * XH5, 11) * XH1;
    h ^= h >> 15;
    h *= XH2;
    h ^= h >> 13;
    h *= XH3;
    h ^= h >> 16;
    return h;
}

// Small host-walked launches (<= kLbFewBlocks blocks, e.g. the range reader's 256 KiB batches):
// one 256-thread workgroup per unit runs the token index (k_dtok's algorithm, all four waves),
// then wave 0 executes the block (k_dexec's) while wave 1 hashes its output from the LDS ring
// (the frame's content xxh32 when the block is the whole frame: blk_hash, which k_dframe_close
// takes instead of hashing again). One launch instead of the large-block path's chain; units it
// does not take are left to k_decode_pe (exact statuses) and get blk_hash 0.
#if !S3HC_SMALL_JUMP  // (the variant: compiled only when selected at build time)
__global__ __launch_bounds__(fst::kTT) void k_dsmall(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                     const DecBlock* __restrict__ blk, const DecUnit* __restrict__ units,
                                                     uint32_t nunits, const uint8_t* __restrict__ unit_lb, FastArgs a,
                                                     uint32_t maxc, uint32_t* __restrict__ blk_out,
                                                     int32_t* __restrict__ blk_status) {
    __shared__ __attribute__((aligned(16))) uint32_t ring[fst::kORW];
    __shared__ uint32_t hsync[2];
    __shared__ DexLds dl;
    const uint32_t wv = threadIdx.x >> 6;
    for (uint32_t u = blockIdx.x; u < nunits; u += gridDim.x) {
        FastUnit F;
        const bool ok = dtok_unit<fst::kTT>(u, src, blk, units, unit_lb, a, maxc, &F);  // (a unit it leaves: bh 0)
        const DecUnit Un = units[u];
        if (!ok) {
            __syncthreads();
            continue;
        }
        if (threadIdx.x == 0) {
            hsync[0] = 0u;
            hsync[1] = 0u;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the records are in memory before the barrier
        __syncthreads();
        if (wv == 0) {
            dexec_unit(u, src, dst, blk, units, blk_out, blk_status, a, F, ring, hsync, &dl);
        } else if (wv == 1) {
            const uint32_t h = hash_ring(ring, hsync, F.U);
            if ((threadIdx.x & 63u) == 0 && a.bh) a.bh[Un.first] = (1ull << 32) | h;
        }
        __syncthreads();
    }
}
#endif  // !S3HC_SMALL_JUMP

// ------------------------------------------------------------------ k_djump
// Small host-walked launches by pointer jumping, for the latency of a few-block batch (the range
// reader's 256 KiB batches) rather than throughput: one 1024-thread workgroup per block indexes it
// (dtok_unit with 1024 speculative segments: records, as k_dtok writes them) and decodes it with
// all 16 waves instead of k_dsmall's one executor wave:
//   positions     the records' output offsets (four per thread, one workgroup scan);
//   pointers      one u16 per output byte in LDS (128 KiB): a literal byte points to itself (and is
//                 copied to the output), a match byte to its source byte (an overlapping match's
//                 bytes to the period before the match), so every pointer leads to a smaller
//                 position until a literal; sequences longer than kShort by the whole workgroup;
//   jumping       P[b] = P[P[b]] in place until no pointer changes (log2 of the longest chain of
//                 rounds: 6 on the bench's log text), eight pointer pairs per thread in flight;
//   output        every dword holding a match byte gathers its bytes from their literals in the
//                 output (one unaligned load when they are consecutive), eight dwords in flight;
//   hash          the block's xxh32 by four lanes (the frame's content checksum: a.bh).
namespace jmp {
constexpr uint32_t kT = 1024;             // threads per workgroup
constexpr uint32_t kQ = 512;              // long sequences written by the whole workgroup
constexpr uint32_t kShort = 64;           // sequence bytes one thread writes alone
constexpr uint32_t kPBytes = 2u * 65536u; // P: u16 per output byte
constexpr uint32_t kLds = kPBytes + 64u;
static_assert(fast_lds_bytes(kFastMaxC) <= kLds, "the staged block fits P's LDS");
}  // namespace jmp

// xxh32 (seed 0) of [p, p + L) in global memory by lanes 0..3 of the calling wave (lane a runs
// accumulator a; 32 stripes of loads in flight ahead of the chain). Valid in lane 0.
#ifndef S3HC_HASH_PRE  // k_djump's block checksum: stripe products (input * PRIME2) by the whole workgroup
#define S3HC_HASH_PRE 1
#endif
// xxh32 of p[0, L) on lanes 0-3 (lane a: accumulator a), with pr[4 s + a] = the stripe words times
// PRIME2 already computed (by the whole workgroup, into LDS): each lane's serial round is then an
// add, a rotate and one multiply
__device__ __forceinline__ uint32_t xxh32_lane4_pre(const uint8_t* __restrict__ p, uint32_t L, const uint32_t* pr) {
    const uint32_t a = threadIdx.x & 3u;
    const uint32_t ns = L >> 4;
    uint32_t acc = a == 0 ? XH1 + XH2 : (a == 1 ? XH2 : (a == 2 ? 0u : 0u - XH1));
    constexpr uint32_t kB = 32;
    uint32_t s = 0;
    for (; s + kB <= ns; s += kB) {
        uint32_t m[kB];
#pragma unroll
        for (uint32_t k = 0; k < kB; ++k) m[k] = pr[4u * (s + k) + a];
#pragma unroll
        for (uint32_t k = 0; k < kB; ++k) acc = xh_rotl(acc + m[k], 13) * XH1;
    }
    for (; s < ns; ++s) acc = xh_rotl(acc + pr[4u * s + a], 13) * XH1;
    const uint32_t v1 = (uint32_t)__shfl((int)acc, 0, 4), v2 = (uint32_t)__shfl((int)acc, 1, 4);
    const uint32_t v3 = (uint32_t)__shfl((int)acc, 2, 4), v4 = (uint32_t)__shfl((int)acc, 3, 4);
    uint32_t h = L >= 16u ? xh_rotl(v1, 1) + xh_rotl(v2, 7) + xh_rotl(v3, 12) + xh_rotl(v4, 18) : XH5;
    h += L;
    uint32_t t = ns * 16u;
    for (; t + 4u <= L; t += 4u) h = xh_rotl(h + gld4(p + t) * XH3, 17) * XH4;
    for (; t < L; ++t) h = xh_rotl(h + (uint32_t)p[t] * XH5, 11) * XH1;
    h ^= h >> 15;
    h *= XH2;
    h ^= h >> 13;
    h *= XH3;
    h ^= h >> 16;
    return h;
}
__device__ __forceinline__ uint32_t xxh32_lane4(const uint8_t* __restrict__ p, uint32_t L) {
    const uint32_t a = threadIdx.x & 3u;
    const uint32_t ns = L >> 4;
    uint32_t acc = a == 0 ? XH1 + XH2 : (a == 1 ? XH2 : (a == 2 ? 0u : 0u - XH1));
    const uint8_t* q = p + 4u * a;  // stripe s: q + 16 s
    constexpr uint32_t kB = 32;
    uint32_t s = 0;
    for (; s + kB <= ns; s += kB) {
        uint32_t m[kB];
#pragma unroll
        for (uint32_t k = 0; k < kB; ++k) m[k] = gld4(q + 16u * (s + k));
#pragma unroll
        for (uint32_t k = 0; k < kB; ++k) acc = xh_round(acc, m[k]);
    }
    for (; s < ns; ++s) acc = xh_round(acc, gld4(q + 16u * s));
    const uint32_t v1 = (uint32_t)__shfl((int)acc, 0, 4), v2 = (uint32_t)__shfl((int)acc, 1, 4);
    const uint32_t v3 = (uint32_t)__shfl((int)acc, 2, 4), v4 = (uint32_t)__shfl((int)acc, 3, 4);
    uint32_t h = L >= 16u ? xh_rotl(v1, 1) + xh_rotl(v2, 7) + xh_rotl(v3, 12) + xh_rotl(v4, 18) : XH5;
    h += L;
    uint32_t t = ns * 16u;
    for (; t + 4u <= L; t += 4u) h = xh_rotl(h + gld4(p + t) * XH3, 17) * XH4;
    for (; t < L; ++t) h = xh_rotl(h + (uint32_t)p[t] * XH5, 11) * XH1;
    h ^= h >> 15;
    h *= XH2;
    h ^= h >> 13;
    h *= XH3;
    h ^= h >> 16;
    return h;
}

// Blocks the token index leaves (stored, malformed, linked, > kFastMaxC compressed) keep bh 0 and
// unit_fast 0 and get their exact statuses from the per-unit decoder: with own_left (a launch of
// one workgroup per unit and no large-block path) this workgroup runs it itself — waves 2-15
// leave the kernel first, so decode_unit_pe's barriers count waves 0-1 only and no barrier of
// this kernel follows; otherwise the per-unit decoder's own launch (k_decode_pe) takes them.
// k_dframe_close closes the frames. (Round 4 also ran the frame close in the last workgroup and
// let waves 2-15 wait at the close's barriers while waves 0-1 were inside the per-unit decoder:
// the barriers paired across code locations, which is the fault of GPUTEST_r04.)
__global__ __launch_bounds__(jmp::kT) void k_djump(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                   const DecBlock* __restrict__ blk, const DecUnit* __restrict__ units,
                                                   uint32_t nunits, const uint8_t* __restrict__ unit_lb, FastArgs a,
                                                   uint32_t maxc, uint32_t* __restrict__ blk_out,
                                                   int32_t* __restrict__ blk_status, uint32_t own_left) {
    using namespace jmp;
    extern __shared__ __attribute__((aligned(16))) uint8_t dsm[];  // (dtok_unit's staged block, then P)
    uint16_t* P = (uint16_t*)dsm;
    uint32_t* P32 = (uint32_t*)dsm;
    __shared__ uint32_t qrec[kQ], qpos[kQ];
    __shared__ uint32_t qn;
    __shared__ uint32_t jscr[32];
    const uint32_t t = threadIdx.x;
    for (uint32_t u = blockIdx.x; u < nunits; u += gridDim.x) {
        FastUnit F;
        // token index and records with all 16 waves (1024 speculative segments)
        if (!dtok_unit<kT>(u, src, blk, units, unit_lb, a, maxc, &F)) {  // (a unit it leaves: bh 0)
            __syncthreads();  // (every thread is done with the staged block)
            if (own_left && gridDim.x >= nunits) {  // (this workgroup's only unit)
                // Invariant this relies on: waves 2-15 end the kernel here, and a workgroup
                // barrier (s_barrier) waits only for the waves of the workgroup that have not
                // ended, so every __syncthreads() inside decode_unit_pe pairs waves 0-1 with
                // each other. That holds because no wave reaches any later barrier of this kernel:
                // waves 0-1 return right after decode_unit_pe, waves 2-15 return now (the
                // GPUTEST_r04 fault was waves waiting at a *different* barrier of the same kernel).
                if (t >= 128u) return;
                decode_unit_pe(u, dsm, src, dst, blk, units, blk_out, blk_status, nullptr, nullptr);
                return;
            }
            continue;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the records are in memory before the barrier
        __syncthreads();
        [[maybe_unused]] const uint64_t tj0 = FP_NOW();
        const DecUnit Un = units[u];
        const DecBlock B = blk[Un.first];
        const uint8_t* in = src + B.src_off;
        uint8_t* out = dst + B.dst_off;
        const uint2* rec = a.rec + B.tok;
        const uint32_t N = F.ntok, U = F.U, C = B.csize;
        if (t == 0) qn = 0u;
        // ---- output positions: thread t's records [t K, t K + K), K <= 11 (N <= kFastMaxTok)
        const uint32_t K = (N + kT - 1u) / kT, r0 = umin_(N, t * K), r1 = umin_(N, r0 + K);
        uint32_t mine = 0;
        {
            uint2 v[4];
            for (uint32_t r = r0; r < r1; r += 4u) {
#pragma unroll
                for (uint32_t e = 0; e < 4u; ++e) v[e] = r + e < r1 ? rec[r + e] : make_uint2(0u, 0u);
#pragma unroll
                for (uint32_t e = 0; e < 4u; ++e) mine += (v[e].x >> 15) + ((v[e].y & 0xFFFFu) ? (v[e].y >> 16) + 4u : 0u);
            }
        }
        uint32_t tot;
        uint32_t o = wg_excl_scan<kT / 64>(mine, jscr, &tot);
        // ---- pointers and literals (sequences longer than kShort: the whole workgroup, below)
        for (uint32_t r = r0; r < r1; ++r) {
            const uint2 v = rec[r];
            const uint32_t ll = v.x >> 15, lit = v.x & 0x7FFFu, off = v.y & 0xFFFFu;
            const uint32_t ml = off ? (v.y >> 16) + 4u : 0u;
            if (ll + ml > kShort) {
                const uint32_t qi = atomicAdd(&qn, 1u);
                if (qi < kQ) {
                    qrec[qi] = r;
                    qpos[qi] = o;
                    o += ll + ml;
                    continue;
                }
            }
            for (uint32_t c = 0; c < ll; c += 16u) {  // (16-byte loads; the block's last bytes bytewise)
                const uint4 x = gld16_blk(in, lit + c, C);
                const uint32_t xw[4] = {x.x, x.y, x.z, x.w}, n = umin_(16u, ll - c);
                for (uint32_t i = 0; i < n; ++i) {
                    out[o + c + i] = (uint8_t)(xw[i >> 2] >> (8u * (i & 3u)));
                    P[o + c + i] = (uint16_t)(o + c + i);
                }
            }
            const uint32_t md = o + ll, ms = md - off;
            if (off >= ml) {
                for (uint32_t i = 0; i < ml; ++i) P[md + i] = (uint16_t)(ms + i);
            } else {
                uint32_t q = 0;
                for (uint32_t i = 0; i < ml; ++i) {
                    P[md + i] = (uint16_t)(ms + q);
                    q = q + 1u == off ? 0u : q + 1u;
                }
            }
            o += ll + ml;
        }
        __syncthreads();
        const uint32_t nq = umin_(qn, kQ);
        for (uint32_t e = 0; e < nq; ++e) {
            const uint2 v = rec[qrec[e]];
            const uint32_t o0 = qpos[e], ll = v.x >> 15, lit = v.x & 0x7FFFu, off = v.y & 0xFFFFu;
            const uint32_t ml = off ? (v.y >> 16) + 4u : 0u;
            for (uint32_t i = t; i < ll; i += kT) {
                out[o0 + i] = in[lit + i];
                P[o0 + i] = (uint16_t)(o0 + i);
            }
            const uint32_t md = o0 + ll, ms = md - off;
            for (uint32_t i = t; i < ml; i += kT) P[md + i] = (uint16_t)(ms + (off >= ml ? i : i % off));
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // literal bytes in memory before the gathers below
        __syncthreads();
        [[maybe_unused]] const uint64_t tj1 = FP_NOW();
        // ---- pointer jumping (pairs of u16 per dword; in place: a pointer read mid-update is an
        // older or newer point of the same chain). kJ pairs per thread at a time: every pair read
        // and every gather of the batch in flight before the first use
        const uint32_t Up = (U + 1u) >> 1;
        [[maybe_unused]] uint32_t nround = 0;
        for (;;) {
            int ch = 0;
            constexpr uint32_t kJ = 8;
            for (uint32_t k0 = t; k0 < Up; k0 += kT * kJ) {
                uint32_t pr[kJ], q[kJ][2];
#pragma unroll
                for (uint32_t e = 0; e < kJ; ++e) {
                    const uint32_t k = k0 + kT * e;
                    pr[e] = k < Up ? P32[k] : 0u;  // (beyond U: pair 0 -> 0, a root)
                }
#pragma unroll
                for (uint32_t e = 0; e < kJ; ++e) {
                    q[e][0] = P[pr[e] & 0xFFFFu];
                    q[e][1] = P[pr[e] >> 16];
                }
#pragma unroll
                for (uint32_t e = 0; e < kJ; ++e) {
                    const uint32_t k = k0 + kT * e;
                    const uint32_t lo = pr[e] & 0xFFFFu, hi = pr[e] >> 16;
                    // a root points to itself (its gather returns it: no change); the odd tail
                    // entry past U is kept as read
                    const uint32_t nlo = q[e][0];
                    const uint32_t nhi = 2u * k + 1u < U ? q[e][1] : hi;
                    if (k < Up && (nlo != lo || nhi != hi)) {
                        P32[k] = nlo | (nhi << 16);
                        ch = 1;
                    }
                }
            }
            ++nround;
            if (!__syncthreads_or(ch)) break;
        }
        [[maybe_unused]] const uint64_t tj2 = FP_NOW();
        // ---- every dword with a match byte: its bytes from their literals, kE dwords per thread
        // at a time (every gather of a batch in flight before its stores)
        const bool al = ((uintptr_t)out & 3u) == 0u;
        constexpr uint32_t kE = 4;
        for (uint32_t b0 = 4u * t; b0 < U; b0 += 4u * kT * kE) {
            uint32_t v[kE], pp[kE][4];
            bool need[kE];
#pragma unroll
            for (uint32_t e = 0; e < kE; ++e) {
                const uint32_t b = b0 + 4u * kT * e;
                const uint32_t n = b < U ? umin_(4u, U - b) : 0u;
                const uint32_t w0 = n ? P32[b >> 1] : 0u, w1 = n ? P32[(b >> 1) + 1u] : 0u;
                pp[e][0] = w0 & 0xFFFFu;
                pp[e][1] = n > 1u ? w0 >> 16 : b + 1u;
                pp[e][2] = n > 2u ? w1 & 0xFFFFu : b + 2u;
                pp[e][3] = n > 3u ? w1 >> 16 : b + 3u;
                need[e] = n && !(pp[e][0] == b && pp[e][1] == b + 1u && pp[e][2] == b + 2u && pp[e][3] == b + 3u);
            }
#pragma unroll
            for (uint32_t e = 0; e < kE; ++e) {
                const uint32_t b = b0 + 4u * kT * e;
                v[e] = 0u;
                if (!need[e]) continue;
                const uint32_t n = umin_(4u, U - b);
                if (n == 4u && pp[e][1] == pp[e][0] + 1u && pp[e][2] == pp[e][0] + 2u && pp[e][3] == pp[e][0] + 3u) {
                    v[e] = gld4(out + pp[e][0]);
                } else {
                    v[e] = (uint32_t)out[pp[e][0]];
                    if (n > 1u) v[e] |= (uint32_t)out[pp[e][1]] << 8;
                    if (n > 2u) v[e] |= (uint32_t)out[pp[e][2]] << 16;
                    if (n > 3u) v[e] |= (uint32_t)out[pp[e][3]] << 24;
                }
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (every gather of the batch before its stores)
#pragma unroll
            for (uint32_t e = 0; e < kE; ++e) {
                const uint32_t b = b0 + 4u * kT * e;
                if (!need[e]) continue;
                const uint32_t n = umin_(4u, U - b);
                if (n == 4u && al) {
                    *(uint32_t*)(out + b) = v[e];
                } else {
                    for (uint32_t i = 0; i < n; ++i) out[b + i] = (uint8_t)(v[e] >> (8u * i));
                }
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        [[maybe_unused]] const uint64_t tj3 = FP_NOW();
#if S3HC_HASH_PRE
        // the stripes' words times PRIME2, by every thread, into LDS over P (no longer needed)
        for (uint32_t i = t; i < (U >> 4) * 4u; i += kT) P32[i] = gld4(out + 4u * i) * XH2;
        __syncthreads();
        if (t < 4u) {
            const uint32_t h = xxh32_lane4_pre(out, U, P32);
#else
        if (t < 4u) {
            const uint32_t h = xxh32_lane4(out, U);
#endif
            if (t == 0) {
                if (a.bh) a.bh[Un.first] = (1ull << 32) | h;
                blk_out[Un.first] = U;
                blk_status[Un.first] = S3HC_OK;
#ifdef FPROF
                const uint64_t tj4 = FP_NOW();
                FP_ADD(25, tj1 - tj0);
                FP_ADD(26, tj2 - tj1);
                FP_ADD(27, tj3 - tj2);
                FP_ADD(28, tj4 - tj3);
                FP_ADD(29, nround);
                FP_ADD(30, 1);
#endif
            }
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------------ k_dexec
// One executor wave per workgroup (k_dtok's records); the frame close hashes the output.
// (<= 128 VGPRs: 4 waves per SIMD, a 4096-block batch resident at once)
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4))) void k_dexec(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                              const DecBlock* __restrict__ blk, const DecUnit* __restrict__ units,
                                              uint32_t nunits, const uint64_t* __restrict__ ucount,
                                              uint32_t* __restrict__ blk_out, int32_t* __restrict__ blk_status,
                                              FastArgs a) {
    const uint32_t nu = unit_count(ucount, nunits);
    __shared__ __attribute__((aligned(16))) uint32_t ring[fst::kORW];
    __shared__ DexLds dl;
    for (uint32_t u = blockIdx.x; u < nu; u += gridDim.x) {
        if (!a.unit_fast[u]) continue;
        dexec_unit(u, src, dst, blk, units, blk_out, blk_status, a, a.fu[u], ring, nullptr, &dl);
        wsync();
    }
}
constexpr uint32_t kDexecUnits = 1, kDexecThreads = 64;
// (the frame close hashes k_dexec's output: a hashing wave beside the executors costs a 4096-block
// batch its one-pass residency)
bool fast_exec_hashes() { return false; }

// ================================================================ launchers
static inline uint32_t fcdiv(uint64_t x, uint64_t y) { return (uint32_t)((x + y - 1) / y); }

hipError_t launch_fast_tok(const uint8_t* src, const DecBlock* blk, const DecUnit* units, uint32_t nunits,
                           const uint64_t* ucount, uint32_t grid, const uint8_t* unit_lb, const FastArgs& a,
                           hipStream_t st) {
    if (!nunits || !grid || !a.maxc) return hipSuccess;
    const uint32_t maxc = a.maxc < kFastMaxC ? a.maxc : kFastMaxC;
    hipLaunchKernelGGL(k_dtok, dim3(grid), dim3(fst::kTT), fast_lds_bytes(maxc), st, src, blk, units, nunits, ucount,
                       unit_lb, a, maxc);
    return hipGetLastError();
}
#ifdef UPROF
extern "C" int s3hc_diag_uprof(unsigned long long* out, int n) {
    if (n > 8192) n = 8192;
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_uprof), sizeof(unsigned long long) * 4 * n) == hipSuccess ? 0 : -1;
}
#endif
#ifdef FPROF
extern "C" int s3hc_diag_fprof(unsigned long long* out, int n, int reset) {
    if (n > 32) n = 32;
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fprof), sizeof(unsigned long long) * n) != hipSuccess) return -1;
    if (reset) {
        unsigned long long z[32] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_fprof), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#endif
// own_left: the launch also decodes the units the fast path leaves (k_djump; no k_decode_pe needed)
hipError_t launch_fast_small(const uint8_t* src, uint8_t* dst, const DecBlock* blk, const DecUnit* units,
                             uint32_t nunits, const uint8_t* unit_lb, const FastArgs& a, uint32_t* blk_out,
                             int32_t* blk_status, hipStream_t st, bool own_left, bool* owned) {
    *owned = false;
    if (!nunits || !a.maxc) return hipSuccess;
    const uint32_t maxc = a.maxc < kFastMaxC ? a.maxc : kFastMaxC;
#if S3HC_SMALL_JUMP
    // > 64 KiB of dynamic LDS: the attribute belongs to the current device, so it is set once per
    // device (a process-wide once would leave every device but the first without it)
    static std::atomic<uint64_t> attr_set{0};
    int dev = 0;
    if (hipError_t e = hipGetDevice(&dev); e != hipSuccess) return e;
    const uint64_t bit = dev < 64 ? 1ull << dev : 0ull;
    if (!bit || !(attr_set.load(std::memory_order_acquire) & bit)) {
        const hipError_t attr = hipFuncSetAttribute((const void*)k_djump, hipFuncAttributeMaxDynamicSharedMemorySize,
                                                    (int)jmp::kLds);
        if (attr != hipSuccess) return attr;
        attr_set.fetch_or(bit, std::memory_order_acq_rel);
    }
    hipLaunchKernelGGL(k_djump, dim3(nunits), dim3(jmp::kT), jmp::kLds, st, src, dst, blk, units, nunits, unit_lb, a,
                       maxc, blk_out, blk_status, own_left ? 1u : 0u);
    *owned = own_left;
#else
    hipLaunchKernelGGL(k_dsmall, dim3(nunits), dim3(fst::kTT), fast_lds_bytes(maxc), st, src, dst, blk, units, nunits,
                       unit_lb, a, maxc, blk_out, blk_status);
#endif
    return hipGetLastError();
}
hipError_t launch_fast_exec(const uint8_t* src, uint8_t* dst, const DecBlock* blk, const DecUnit* units,
                            uint32_t nunits, const uint64_t* ucount, uint32_t grid, uint32_t* blk_out,
                            int32_t* blk_status, const FastArgs& a, hipStream_t st) {
    if (!nunits || !grid) return hipSuccess;
    hipLaunchKernelGGL(k_dexec, dim3((grid + kDexecUnits - 1u) / kDexecUnits), dim3(kDexecThreads), 0, st, src, dst,
                       blk, units, nunits, ucount, blk_out, blk_status, a);
    return hipGetLastError();
}
}  // namespace s3hc
