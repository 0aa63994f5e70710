// s3hc_kernels.hip — CDNA4 (gfx950) kernels of the LZ4 frame engine.
//
// Everything here is integer byte work on 64-lane waves; none of it is GEMM-shaped,
// so there is no MFMA. The kernels are:
//   k_xxh32_ranges   xxh32 (twox-hash XxHash32, compression.rs:35/364) of many byte ranges;
//                    4 lanes per range, one per XXH32 accumulator chain.
//   k_decode_units   LZ4 block decode (lz4_flex FrameDecoder semantics, compression.rs:479-480):
//                    one wave per unit; wave-speculative token parsing over 64 candidate
//                    positions, an LDS ring of recent output for match sources, coalesced
//                    1 KiB flushes to HBM.
//   k_enc_parse      LZ4 match finding: one wave per 4 KiB segment, per-wave LDS hash table,
//                    64 positions probed per step, ballot picks the first match (greedy).
//   k_enc_sizes      per block: merges segment carries, sizes the payload, picks stored vs
//                    compressed exactly like lz4_flex write_block (comp_len < src_len).
//   k_enc_emit       one wave per segment: writes frame header, block word, tokens,
//                    literals, offsets, EndMark and content checksum (compression.rs:326-368
//                    byte layout for stored blocks).
//   k_dframe_*       device-side frame walk for device-resident batches.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "s3hc_plan.hpp"
#include "s3hc_knobs.hpp"
#include "s3hc_lz4.h"

namespace s3hc {

// ------------------------------------------------------------------ helpers
__device__ __forceinline__ uint32_t rotl32(uint32_t x, int r) {
    return __builtin_amdgcn_alignbit(x, x, 32 - r);
}
__device__ __forceinline__ uint32_t rdl(uint32_t v, uint32_t l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l);
}
__device__ __forceinline__ int lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0)); }

// Serial scalar walks (one readlane per hop) raise the wave's issue priority so their
// readlanes are not queued behind other waves' vector work (diagnostic builds can disable).
#ifndef S3HC_WALK_PRIO
#define S3HC_WALK_PRIO 3
#endif
#define WALK_PRIO_ON() __builtin_amdgcn_s_setprio(S3HC_WALK_PRIO)
#define WALK_PRIO_OFF() __builtin_amdgcn_s_setprio(0)

// Orders this wave's LDS traffic across lanes (lanes of one wave share an in-order LDS queue;
// this only stops the compiler from moving accesses across the point).
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Phase timers for diagnostic builds only (S3HC_DIAG_LEVEL 10): per-wave s_memtime sums into
// g_prof, read back with s3hc_diag_prof. Compiled out of the shipped library.
#if defined(S3HC_DIAG_LEVEL) && S3HC_DIAG_LEVEL == 10
#define S3HC_PROF 1
__device__ unsigned long long g_prof[32];
#define PROF_NOW() __builtin_amdgcn_s_memtime()
#define PROF_ADD(arr, k, v) (arr)[k] += (v)
#else
#define PROF_NOW() 0ull
#define PROF_ADD(arr, k, v) ((void)(v))
#endif

// 4 bytes at any LDS byte offset: two aligned dword reads + v_alignbyte.
__device__ __forceinline__ uint32_t lds32u(const uint8_t* lds, uint32_t i) {
    const uint32_t* w = (const uint32_t*)(lds + (i & ~3u));
    return __builtin_amdgcn_alignbyte(w[1], w[0], i & 3u);
}

// 4 bytes at any global address where `avail` (>= 1) bytes from p are valid. Only aligned
// dwords that contain a valid byte are touched (never faults past the end of a buffer).
__device__ __forceinline__ uint32_t gld32u(const uint8_t* p, uint32_t avail) {
    uintptr_t a = (uintptr_t)p;
    const uint32_t* w = (const uint32_t*)(a & ~(uintptr_t)3);
    uint32_t sh = (uint32_t)(a & 3);
    uint32_t lo = w[0];
    uint32_t hi = (sh != 0 && avail > 4 - sh) ? w[1] : 0u;
    return __builtin_amdgcn_alignbyte(hi, lo, sh);
}

// DPP lane moves (GFX9 row_shr / row_bcast): lanes without a source read 0.
template <int CTRL, int ROWMASK>
__device__ __forceinline__ uint32_t dpp0(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROWMASK, 0xF, false);
}
// Inclusive wave-wide sum / max (Hillis-Steele inside 16-lane rows, then row broadcasts).
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t x) {
    x += dpp0<0x111, 0xF>(x);
    x += dpp0<0x112, 0xF>(x);
    x += dpp0<0x114, 0xF>(x);
    x += dpp0<0x118, 0xF>(x);
    x += dpp0<0x142, 0xA>(x);
    x += dpp0<0x143, 0xC>(x);
    return x;
}
__device__ __forceinline__ uint32_t umax32(uint32_t a, uint32_t b) { return a > b ? a : b; }
__device__ __forceinline__ uint32_t umin32(uint32_t a, uint32_t b) { return a < b ? a : b; }
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t x) {
    x = umax32(x, dpp0<0x111, 0xF>(x));
    x = umax32(x, dpp0<0x112, 0xF>(x));
    x = umax32(x, dpp0<0x114, 0xF>(x));
    x = umax32(x, dpp0<0x118, 0xF>(x));
    x = umax32(x, dpp0<0x142, 0xA>(x));
    x = umax32(x, dpp0<0x143, 0xC>(x));
    return x;
}
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v, int) { return wave_incl_sum(v) - v; }
template <int CTRL, int ROWMASK>
__device__ __forceinline__ uint64_t dpp0_64(uint64_t x) {
    return (uint64_t)dpp0<CTRL, ROWMASK>((uint32_t)(x >> 32)) << 32 | dpp0<CTRL, ROWMASK>((uint32_t)x);
}
__device__ __forceinline__ uint64_t wave_incl_sum64(uint64_t x) {
    x += dpp0_64<0x111, 0xF>(x);
    x += dpp0_64<0x112, 0xF>(x);
    x += dpp0_64<0x114, 0xF>(x);
    x += dpp0_64<0x118, 0xF>(x);
    x += dpp0_64<0x142, 0xA>(x);
    x += dpp0_64<0x143, 0xC>(x);
    return x;
}

// Wave-cooperative copy of n bytes global -> global, any alignment of either side.
// Loads for up to 4 KiB are issued before the stores.
__device__ void wave_copy_global(uint8_t* dst, const uint8_t* src, uint32_t n, int lane) {
    uintptr_t da = (uintptr_t)dst;
    uint32_t head = (uint32_t)((16 - (da & 15)) & 15);
    if (head > n) head = n;
    if ((uint32_t)lane < head) dst[lane] = src[lane];
    const uint32_t nv = (n - head) >> 4;
    const uint8_t* s = src + head;
    uint8_t* d = dst + head;
    const uintptr_t sa = (uintptr_t)s;
    const uint32_t sh = (uint32_t)(sa & 3);
    const uint32_t* sw = (const uint32_t*)(sa & ~(uintptr_t)3);
    for (uint32_t base = 0; base < nv; base += 64 * 2) {
        const uint32_t ja = base + lane, jb = base + lane + 64;
        const uint32_t ka = ja < nv ? ja : nv - 1, kb = jb < nv ? jb : nv - 1;
        uint4 va, vb;
        if (sh == 0) {
            va = make_uint4(sw[4 * ka], sw[4 * ka + 1], sw[4 * ka + 2], sw[4 * ka + 3]);
            vb = make_uint4(sw[4 * kb], sw[4 * kb + 1], sw[4 * kb + 2], sw[4 * kb + 3]);
        } else {
            const uint32_t a0 = sw[4 * ka], a1 = sw[4 * ka + 1], a2 = sw[4 * ka + 2], a3 = sw[4 * ka + 3], a4 = sw[4 * ka + 4];
            const uint32_t b0 = sw[4 * kb], b1 = sw[4 * kb + 1], b2 = sw[4 * kb + 2], b3 = sw[4 * kb + 3], b4 = sw[4 * kb + 4];
            va = make_uint4(__builtin_amdgcn_alignbyte(a1, a0, sh), __builtin_amdgcn_alignbyte(a2, a1, sh),
                            __builtin_amdgcn_alignbyte(a3, a2, sh), __builtin_amdgcn_alignbyte(a4, a3, sh));
            vb = make_uint4(__builtin_amdgcn_alignbyte(b1, b0, sh), __builtin_amdgcn_alignbyte(b2, b1, sh),
                            __builtin_amdgcn_alignbyte(b3, b2, sh), __builtin_amdgcn_alignbyte(b4, b3, sh));
        }
        if (ja < nv) *(uint4*)(d + 16 * ja) = va;
        if (jb < nv) *(uint4*)(d + 16 * jb) = vb;
    }
    for (uint32_t t = head + 16 * nv + (uint32_t)lane; t < n; t += 64) dst[t] = src[t];
}

// Wave-cooperative store of n bytes from (contiguous) LDS to global, any global alignment.
__device__ void wave_store_from_lds(uint8_t* dst, const uint8_t* lds, uint32_t n, int lane) {
    uintptr_t da = (uintptr_t)dst;
    uint32_t head = (uint32_t)((16 - (da & 15)) & 15);
    if (head > n) head = n;
    if ((uint32_t)lane < head) dst[lane] = lds[lane];
    uint32_t body = (n - head) & ~15u;
    for (uint32_t c = (uint32_t)lane * 16; c < body; c += 64 * 16) {
        uint32_t i = head + c;
        uint4 v = make_uint4(lds32u(lds, i), lds32u(lds, i + 4), lds32u(lds, i + 8), lds32u(lds, i + 12));
        *(uint4*)(dst + i) = v;
    }
    for (uint32_t t = head + body + (uint32_t)lane; t < n; t += 64) dst[t] = lds[t];
}

// ------------------------------------------------------------------- xxh32
#define XP1 2654435761U
#define XP2 2246822519U
#define XP3 3266489917U
#define XP4 668265263U
#define XP5 374761393U

__device__ __forceinline__ uint32_t xround(uint32_t acc, uint32_t in) {
    acc += in * XP2;
    acc = rotl32(acc, 13);
    return acc * XP1;
}

// xxh32 of [p, p + L) by the 4 lanes 4k..4k+3 of a wave (a = lane & 3 picks the accumulator);
// every lane calls (shuffles), the result is valid in lane a == 0 of an active group.
template <uint32_t kIF, bool kPipe>  // loads per batch (VGPRs: the match finder's copy uses fewer)
__device__ __forceinline__ uint32_t xxh32_lanes(const uint8_t* __restrict__ p, uint32_t L, bool act, uint32_t a) {
    const int lane = lane_id();
    const uint32_t ns = L >> 4;
    uint32_t acc = a == 0 ? XP1 + XP2 : (a == 1 ? XP2 : (a == 2 ? 0u : 0u - XP1));
    const uint8_t* q = p + 4 * a;
    uint32_t s = 0;
    if (kPipe && (((uintptr_t)p) & 3) == 0) {
        // software-pipelined: three buffers of kIF stripes, the loads of the next two in flight
        // while one is hashed (the chain add, rotate, multiply is the only serial part)
        const uint32_t* w = (const uint32_t*)q;
        uint32_t b0[kIF], b1[kIF], b2[kIF];
        const uint32_t nbt = ns / kIF;
#define XLD(buf, bidx)                                                        \
    {                                                                         \
        const uint32_t bb_ = (bidx) < nbt ? (bidx) : 0u;                      \
        _Pragma("unroll") for (uint32_t k = 0; k < kIF; ++k) buf[k] = w[4 * (bb_ * kIF + k)]; \
    }
#define XUSE(buf) _Pragma("unroll") for (uint32_t k = 0; k < kIF; ++k) acc = xround(acc, buf[k]);
        XLD(b0, 0u)
        XLD(b1, 1u)
        for (uint32_t b = 0; b < nbt; b += 3) {
            XLD(b2, b + 2)
            XUSE(b0)
            XLD(b0, b + 3)
            if (b + 1 < nbt) { XUSE(b1) }
            XLD(b1, b + 4)
            if (b + 2 < nbt) { XUSE(b2) }
        }
#undef XLD
#undef XUSE
        for (s = nbt * kIF; s < ns; ++s) acc = xround(acc, w[4 * s]);
    } else if ((((uintptr_t)p) & 3) == 0) {
        const uint32_t* w = (const uint32_t*)q;
        // kIF loads in flight per lane: the chain (add, rotate, multiply) is the only serial part
        for (; s + kIF <= ns; s += kIF) {
            uint32_t v[kIF];
#pragma unroll
            for (uint32_t k = 0; k < kIF; ++k) v[k] = w[4 * (s + k)];
#pragma unroll
            for (uint32_t k = 0; k < kIF; ++k) acc = xround(acc, v[k]);
        }
        for (; s < ns; ++s) acc = xround(acc, w[4 * s]);
    } else {
        for (; s < ns; ++s) acc = xround(acc, gld32u(q + 16 * s, L - 16 * s - 4 * a));
    }
    const int qb = lane & ~3;
    uint32_t v1 = __shfl(acc, qb), v2 = __shfl(acc, qb + 1), v3 = __shfl(acc, qb + 2), v4 = __shfl(acc, qb + 3);
    if (!act || a != 0) return 0u;
    uint32_t h = L >= 16 ? rotl32(v1, 1) + rotl32(v2, 7) + rotl32(v3, 12) + rotl32(v4, 18) : XP5;
    h += L;
    uint32_t t = ns * 16;
    while (t + 4 <= L) {
        h += gld32u(p + t, L - t) * XP3;
        h = rotl32(h, 17) * XP4;
        t += 4;
    }
    while (t < L) {
        h += (uint32_t)p[t] * XP5;
        h = rotl32(h, 11) * XP1;
        t++;
    }
    h ^= h >> 15;
    h *= XP2;
    h ^= h >> 13;
    h *= XP3;
    h ^= h >> 16;
    return h;
}

// out[r] = xxh32(base + off[r], len[r], seed 0). Lanes 4r..4r+3 run the 4 accumulator chains
// (gid = global thread index of the calling grid's xxh32 threads).
template <uint32_t kIF, bool kPipe>
__device__ __forceinline__ void xxh32_ranges_dev(const uint8_t* __restrict__ base, const uint64_t* __restrict__ off,
                                                 const uint32_t* __restrict__ len, uint32_t n,
                                                 uint32_t* __restrict__ out, uint32_t gid) {
    const uint32_t r = gid >> 2, a = gid & 3;
    const bool act = r < n;
    const uint32_t L = act ? len[r] : 0u;
    const uint32_t h = xxh32_lanes<kIF, kPipe>(base + (act ? off[r] : 0), L, act, a);
    if (act && a == 0) out[r] = h;
}
__global__ __launch_bounds__(64) void k_xxh32_ranges(const uint8_t* __restrict__ base,
                                                      const uint64_t* __restrict__ off,
                                                      const uint32_t* __restrict__ len, uint32_t n,
                                                      uint32_t* __restrict__ out) {
    xxh32_ranges_dev<32, true>(base, off, len, n, out, blockIdx.x * blockDim.x + threadIdx.x);
}

// ================================================================== decode
namespace dec {
constexpr uint32_t kCring = 2048;  // compressed input ring per wave (aligned-address space)
constexpr uint32_t kCmask = kCring - 1;
constexpr uint32_t kChunk = 256;   // ring refill granule: one dword per lane
constexpr uint32_t kAhead = 1024;  // input kept staged ahead of the parse position
constexpr uint32_t kInit = 5;      // chunks loaded up front (>= kAhead + 3 bytes)
#ifndef S3HC_DEC_PK
#define S3HC_DEC_PK 4
#endif
constexpr uint32_t kPK = S3HC_DEC_PK;  // token positions per lane and window
constexpr uint32_t kPos = 64 * kPK;    // token positions examined per window
constexpr uint32_t kMaxMem = 128;  // members (sequences) per window
constexpr uint32_t kRing = 4096;   // recent output kept in LDS per wave (match sources)
constexpr uint32_t kMask = kRing - 1;
constexpr uint32_t kFlush = 1024;  // ring -> HBM flush granule
constexpr uint32_t kWin = 1024;    // output bytes executed per window (byte-parallel)
constexpr uint32_t kMarks = 1280;  // marks entries: >= kWin + 3 rounded up to the 256-byte pass
constexpr uint32_t kRefs = 256;    // refs entries: one 256-byte pass
constexpr uint32_t kSink = 64;     // per-lane store sink for lanes with nothing to store
[[maybe_unused]] constexpr uint32_t kWaveLds = kRing + kCring + kMarks + 2 * kRefs + kSink + kMaxMem * 8;
[[maybe_unused]] constexpr int kWaves = 4;  // (one-wave decoder: S3HC_DIAG_VARIANTS builds)
enum : uint32_t { F_ERR = 1, F_LAST = 2, F_LONG = 4, F_MORE = 8 };
static_assert(kInit * kChunk >= kAhead + 3, "initial stage must cover the look-ahead");
static_assert(kMaxMem <= 255, "marks hold member index + 1 in a byte");
}  // namespace dec

struct DecWave {
    uint8_t* ring;
    uint8_t* cin;        // kCring bytes: compressed input, byte p of the block at (p + mis) & kCmask
    uint8_t* marks;      // kMarks bytes: sequence start marks of the current window (zero between windows)
    uint16_t* refs;      // kRefs entries: in-pass match source of each output byte of the current pass
    uint8_t* sink;       // kSink bytes: target of stores from lanes with nothing to store
    uint2* mtab;         // the window's member sequences (start, ll, off, literal)
    uint32_t mmax;       // last valid mtab index
    uint8_t* out;        // unit output base in HBM
#ifdef S3HC_PROF
    uint64_t pr[16];
#endif
    uint32_t upos;       // bytes produced in this unit
    uint32_t flushed;    // bytes of the unit already written to HBM
    int lane;
};

__device__ __forceinline__ void dec_flush(DecWave& w, uint32_t from, uint32_t n) {
    // [from, from+n) is contiguous in the ring (from is a multiple of kFlush or n < kFlush
    // and the range does not wrap) -> HBM.
    const uint8_t* src = w.ring + (from & dec::kMask);
    uint8_t* dst = w.out + from;
    if ((((uintptr_t)dst) & 15) == 0 && n == dec::kFlush) {
        uint4 v = *(const uint4*)(src + 16 * w.lane);
        *(uint4*)(dst + 16 * w.lane) = v;
    } else {
        wave_store_from_lds(dst, src, n, w.lane);
    }
}
__device__ __forceinline__ void dec_maybe_flush(DecWave& w) {
    while (w.upos - w.flushed >= dec::kFlush) {
        dec_flush(w, w.flushed, dec::kFlush);
        w.flushed += dec::kFlush;
    }
}
__device__ __forceinline__ void dec_final_flush(DecWave& w) {
    dec_maybe_flush(w);
    uint32_t rem = w.upos - w.flushed;
    if (rem) {
        uint32_t first = dec::kRing - (w.flushed & dec::kMask);
        if (rem <= first) {
            dec_flush(w, w.flushed, rem);
        } else {
            dec_flush(w, w.flushed, first);
            dec_flush(w, w.flushed + first, rem - first);
        }
        w.flushed = w.upos;
    }
}

// Literal run [lit, lit+ll) of the block input -> output (from the input ring when staged).
__device__ __forceinline__ void dec_literals(DecWave& w, const uint8_t* in, uint32_t lit, uint32_t ll,
                                             uint32_t mis, bool staged) {
    for (uint32_t k0 = 0; k0 < ll; k0 += 64) {
        uint32_t piece = ll - k0 < 64 ? ll - k0 : 64;
        uint32_t base = w.upos;
        if ((uint32_t)w.lane < piece) {
            uint32_t k = k0 + w.lane;
            uint8_t b = staged ? w.cin[(lit + k + mis) & dec::kCmask] : in[lit + k];
            w.ring[(base + w.lane) & dec::kMask] = b;
        }
        w.upos = base + piece;
        dec_maybe_flush(w);
    }
}

// Match of ml bytes at distance off (off validated by the caller).
__device__ __forceinline__ void dec_match(DecWave& w, uint32_t off, uint32_t ml) {
    const uint32_t p = w.upos;
    for (uint32_t k0 = 0; k0 < ml; k0 += 64) {
        uint32_t piece = ml - k0 < 64 ? ml - k0 : 64;
        uint32_t base = w.upos;
        if ((uint32_t)w.lane < piece) {
            uint32_t k = k0 + w.lane;
            uint32_t x = off >= ml ? p - off + k : p - off + (k % off);
            uint8_t b;
            if (x + (dec::kRing - 64) >= base) b = w.ring[x & dec::kMask];
            else b = w.out[x];  // older than the ring: already flushed by this wave
            w.ring[(base + w.lane) & dec::kMask] = b;
        }
        w.upos = base + piece;
        dec_maybe_flush(w);
    }
}

// 4 bytes at aligned-space index i of the input ring (wraps).
__device__ __forceinline__ uint32_t cin32(const uint8_t* cin, uint32_t i) {
    const uint32_t* r = (const uint32_t*)cin;
    const uint32_t a = i >> 2;
    return __builtin_amdgcn_alignbyte(r[(a + 1) & (dec::kCring / 4 - 1)], r[a & (dec::kCring / 4 - 1)], i & 3u);
}

// The same read for rings followed by a mirror of their first dword (k_decode_pe): one mask,
// one ds_read2_b32, one alignbyte.
template <bool kMir>
__device__ __forceinline__ uint32_t cin32m(const uint8_t* cin, uint32_t i) {
    if (!kMir) return cin32(cin, i);
    const uint32_t a = i & dec::kCmask;
    const uint32_t* r = (const uint32_t*)(cin + (a & ~3u));
    return __builtin_amdgcn_alignbyte(r[1], r[0], a & 3u);
}

// Wave-cooperative LZ4 length-extension scan at pos (bytes of 255 continue the run).
__device__ __forceinline__ int dec_ext_scan(const uint8_t* in, uint32_t C, uint32_t& pos, uint32_t& acc, int lane) {
    for (;;) {
        uint32_t k = pos + lane;
        uint32_t b = k < C ? (uint32_t)in[k] : 0x100u;
        uint64_t m = __ballot(b != 255u);
        if (m == 0) {
            acc += 255u * 64u;
            pos += 64;
            if (acc > (64u << 20)) return S3HC_CORRUPT;
            continue;
        }
        uint32_t f = (uint32_t)__builtin_ctzll(m);
        uint32_t bf = rdl(b, f);
        if (bf == 0x100u) return S3HC_CORRUPT;
        acc += 255u * f + bf;
        pos += f + 1;
        return S3HC_OK;
    }
}

// One sequence executed wave-wide (literal run, then match unless `last`), with the lz4_flex
// bound checks in stream order. Used for sequences too long for a window.
__device__ __forceinline__ int dec_seq(DecWave& w, const uint8_t* in, uint32_t lit, uint32_t ll, bool last,
                                       uint32_t off, uint32_t ml, uint32_t mis, uint32_t fill, uint32_t bstart,
                                       uint32_t limit, uint32_t cap, uint32_t hist) {
    const uint32_t produced = w.upos - bstart;
    if (ll > limit - produced) return S3HC_CORRUPT;
    if (ll > cap - produced) return S3HC_DST_TOO_SMALL;
    dec_literals(w, in, lit, ll, mis, lit + ll + mis <= fill);  // lit >= the parse position
    if (last) return S3HC_OK;
    const uint32_t have = w.upos - bstart;
    if (off == 0 || off > have + hist) return S3HC_CORRUPT;
    if (ml > limit - have) return S3HC_CORRUPT;
    if (ml > cap - have) return S3HC_DST_TOO_SMALL;
    dec_match(w, off, ml);
    return S3HC_OK;
}

// Byte-parallel execution of one window's sequences (members: lanes of set 0/1; S output
// bytes, S <= kWin). Passes of 256 output bytes, 4 consecutive bytes per lane (one aligned
// ring dword): each byte finds its sequence (start marks + DPP max-scan; a lane's 4 bytes
// touch at most 2 sequences), literal bytes and match bytes whose source precedes this pass
// are read at once, the dword is merged and stored, and bytes whose source lies in this pass
// follow the chain of in-pass sources (refs) to a byte already final. A fixed handful of LDS
// round trips per 256 bytes, almost no scalar work.
__device__ __forceinline__ void dec_window_passes(DecWave& w, uint32_t S, bool far);
__device__ __forceinline__ void dec_window_exec(DecWave& w, uint32_t S, bool isM0, bool isM1, uint32_t orel0,
                                                uint32_t orel1, uint32_t sl0, uint32_t sl1, uint32_t ll0,
                                                uint32_t ll1, uint32_t off0, uint32_t off1, uint32_t lr0,
                                                uint32_t lr1) {
    using namespace dec;
    const int lane = w.lane;
    const uint32_t upos = w.upos;
    const uint32_t a0 = upos & 3u;
    // member m starts at window byte orel: marks[orel + a0] = m + 1 (marks are zero between
    // windows: each pass clears the dwords it reads). The member table holds
    // (M | E << 16, L | off << 16): M = window byte where the member's match starts (orel + ll),
    // E = M + off (saturated; bytes at or past E copy an overlapping match), L = literal ring
    // index minus orel (window byte t of a literal run is cin[(L + t) & kCmask]).
    *((isM0 && sl0) ? w.marks + orel0 + a0 : w.sink + lane) = (uint8_t)(lane + 1);
    *((isM1 && sl1) ? w.marks + orel1 + a0 : w.sink + lane) = (uint8_t)(lane + 65);
    auto entry = [](uint32_t orel, uint32_t ll, uint32_t off, uint32_t lr) -> uint2 {
        const uint32_t M = orel + ll;
        const uint32_t E = M + off < 0xFFFFu ? M + off : 0xFFFFu;
        return make_uint2(M | (E << 16), ((lr - orel) & 0xFFFFu) | (off << 16));
    };
    w.mtab[lane] = entry(orel0, ll0, off0, lr0);
    w.mtab[64 + lane] = entry(orel1, ll1, off1, lr1);
    // a source older than the ring (read back from HBM) needs a match offset above kRing - S
    const bool far = (upos > kRing - S) &&
                     __ballot((isM0 && sl0 > ll0 && off0 > kRing - S) || (isM1 && sl1 > ll1 && off1 > kRing - S));
    dec_window_passes(w, S, far);
}

// The byte-parallel passes of one window whose marks and member table (w.mtab, w.mmax
// entries) are in LDS.
__device__ __forceinline__ void dec_window_passes(DecWave& w, uint32_t S, bool far) {
    using namespace dec;
    const int lane = w.lane;
    uint8_t* marks = w.marks;
    uint16_t* refs = w.refs;
    const uint32_t upos = w.upos;
    const uint32_t a0 = upos & 3u;        // byte u of a pass = window byte u - a0 (ring dwords aligned)
    const uint32_t xbase = upos - a0;
    const uint32_t np = (S + a0 + 255u) >> 8;
    wave_sync();
    uint32_t carry = 0;
    for (uint32_t p = 0; p < np; ++p) {
        const uint32_t u0 = 256u * p + 4u * (uint32_t)lane;  // marks/refs index of this lane's byte 0
        const uint32_t t0 = u0 - a0;                         // window byte of byte 0 (may wrap below 0)
        const uint32_t X = xbase + u0;                        // output position of byte 0 (4-aligned)
        const uint32_t brc = p ? 256u * p - a0 : 0u;          // first window byte of this pass
        // ---- owners
        const uint32_t md = ((const uint32_t*)marks)[64u * p + (uint32_t)lane];
        ((uint32_t*)marks)[64u * p + (uint32_t)lane] = 0u;
        const uint32_t b0 = md & 0xFFu, b1 = (md >> 8) & 0xFFu, b2 = (md >> 16) & 0xFFu, b3 = md >> 24;
        const uint32_t c1 = umax32(b0, b1), c2 = umax32(c1, b2), c3 = umax32(c2, b3);
        const uint32_t inc = wave_incl_max(c3);
        const uint32_t ex = umax32(dpp0<0x138, 0xF>(inc), carry);  // wave_shr:1 -> exclusive
        carry = umax32(carry, rdl(inc, 63));
        uint32_t o[4];
        o[0] = umax32(ex, b0);
        o[1] = umax32(ex, c1);
        o[2] = umax32(ex, c2);
        o[3] = umax32(ex, c3);
        const uint2 fA = w.mtab[umin32(o[0] - 1u, w.mmax)], fB = w.mtab[umin32(o[3] - 1u, w.mmax)];
        // ---- sources
        uint32_t y[4], ci[4], mst[4], mf[4];
        bool lit[4], ok[4], wrap[4];
        bool anywrap = false;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const bool useB = o[j] == o[3];
            const uint32_t fx = useB ? fB.x : fA.x, fy = useB ? fB.y : fA.y;
            const uint32_t t = t0 + j;        // window byte
            mst[j] = fx & 0xFFFFu;            // match start of the owner
            mf[j] = fy >> 16;                 // match offset
            ok[j] = t < S;
            lit[j] = t < mst[j];
            wrap[j] = ok[j] & (t >= (fx >> 16));  // inside an overlapping match
            anywrap |= wrap[j];
            ci[j] = (fy + t) & kCmask;        // literal ring index (carries out of the low half drop)
            y[j] = X + j - mf[j];             // non-overlapping source
        }
        if (__ballot(anywrap)) {
            // overlapping matches (period moff): the source is the byte ee mod moff of the first
            // period. ee < kWin and moff < ee, so ee * rcp(moff) is within 2^-11 of ee / moff and
            // its truncation is exact or one short (at exact multiples), fixed by one compare.
            const float rA = __builtin_amdgcn_rcpf((float)(fA.y >> 16));
            const float rB = __builtin_amdgcn_rcpf((float)(fB.y >> 16));
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (wrap[j]) {
                    const uint32_t ee = t0 + j - mst[j];  // position inside the match
                    const float rf = o[j] == o[3] ? rB : rA;
                    const uint32_t qt = (uint32_t)((float)ee * rf);
                    uint32_t rm = ee - __umul24(qt, mf[j]);
                    rm = rm >= mf[j] ? rm - mf[j] : rm;
                    y[j] = X + j - ee - mf[j] + rm;
                }
            }
        }
        // Sources older than the ring (offsets above kRing - S; a third of log-text matches) are
        // read back from HBM, where this wave flushed them windows ago. All four loads are issued
        // at once, before the LDS reads, and merged into the ring dword before its store: one
        // round trip per pass instead of four serialized load + vmcnt(0) waits.
        uint32_t fv = 0, fmask = 0;
        bool anyold = false;
        if (far) {
            bool old[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                old[j] = ok[j] & !lit[j] & (y[j] < upos - (kRing - S));
                anyold |= old[j];
            }
            if (__ballot(anyold)) {
                uint32_t fb[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) fb[j] = w.out[old[j] ? y[j] : 0u];  // unit byte 0: always valid
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    fv |= old[j] ? fb[j] << (8 * j) : 0u;
                    fmask |= old[j] ? 0xFFu << (8 * j) : 0u;
                }
            }
        }
        const uint32_t oldw = ((const uint32_t*)w.ring)[(X & kMask) >> 2];
        uint32_t v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint8_t* a = lit[j] ? w.cin + ci[j] : w.ring + (y[j] & kMask);
            v[j] = *a;
        }
        bool pnd[4];
        bool anypnd = false;
        uint32_t vm = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t ry = y[j] - upos;  // window byte of the source (< S: inside the window)
            pnd[j] = ok[j] & !lit[j] & (ry - brc < S - brc);  // earlier passes are final in the ring
            anypnd |= pnd[j];
            vm |= ok[j] ? 0xFFu << (8 * j) : 0u;
        }
        const uint32_t val = ((v[0] | (v[1] << 8) | (v[2] << 16) | (v[3] << 24)) & ~fmask) | fv;
        ((uint32_t*)w.ring)[(X & kMask) >> 2] = (val & vm) | (oldw & ~vm);
#ifdef S3HC_PROF
        const uint64_t tq0 = PROF_NOW();
#endif
        if (__ballot(anypnd)) {
            // sources inside this pass: follow refs through pending bytes (bytes of earlier
            // passes and bytes with refs == 0xFFFF are final in the ring); refs are pass-local
            // and written only when some byte of the pass needs them
            const uint32_t r0 = pnd[0] ? y[0] - upos : 0xFFFFu, r1 = pnd[1] ? y[1] - upos : 0xFFFFu;
            const uint32_t r2 = pnd[2] ? y[2] - upos : 0xFFFFu, r3 = pnd[3] ? y[3] - upos : 0xFFFFu;
            *(uint2*)(refs + 4u * (uint32_t)lane) = make_uint2(r0 | (r1 << 16), r2 | (r3 << 16));
            wave_sync();
            uint32_t z[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) z[j] = pnd[j] ? y[j] - upos : brc;
            for (;;) {
                bool more = false;
                uint32_t r[4];
                // refs index of window byte z in this pass: z + a0 - 256p (in [0, 256) for z >= brc)
#pragma unroll
                for (int j = 0; j < 4; ++j) r[j] = refs[(z[j] + a0 - 256u * p) & (kRefs - 1u)];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const bool mo = pnd[j] & (z[j] >= brc) & (r[j] != 0xFFFFu);
                    z[j] = mo ? r[j] : z[j];
                    more |= mo;
                }
                if (!__ballot(more)) break;
            }
            uint8_t vv[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) vv[j] = w.ring[(upos + z[j]) & kMask];
#pragma unroll
            for (int j = 0; j < 4; ++j) *(pnd[j] ? w.ring + ((X + j) & kMask) : w.sink + lane) = vv[j];
        }
        wave_sync();
#ifdef S3HC_PROF
        __builtin_amdgcn_s_waitcnt(0);
        PROF_ADD(w.pr, 14, PROF_NOW() - tq0);
        PROF_ADD(w.pr, 15, __ballot(anyold) ? 1 : 0);
#endif
    }
    w.upos = upos + S;
    const uint64_t tf = PROF_NOW();
    dec_maybe_flush(w);
    PROF_ADD(w.pr, 10, PROF_NOW() - tf);
}

// Speculative LZ4 token parse at block position qq (the window assumes a token there): two
// LDS round trips (token + up to two length bytes; offset + up to two match-length bytes),
// no branches. Flags: F_ERR malformed, F_LAST last sequence, F_LONG a length run beyond two
// bytes, F_MORE bytes past the staged input (both go to the slow path).
struct DecTok {
    uint32_t flags, nxt, lit, ll, off, ml;
};
template <bool kMir = false>
__device__ __forceinline__ DecTok dec_spec(const uint8_t* cin, uint32_t qq, uint32_t mis, uint32_t C, uint32_t fill) {
    using namespace dec;
    DecTok T;
    const uint32_t i = qq + mis;
    const uint32_t w0 = cin32m<kMir>(cin, i);
    const uint32_t t = w0 & 0xFFu, L = t >> 4, M = t & 15u;
    const uint32_t e1 = (w0 >> 8) & 0xFFu, e2 = (w0 >> 16) & 0xFFu;
    const uint32_t x1 = L == 15u ? 1u : 0u, x2 = (L == 15u && e1 == 255u) ? 1u : 0u;
    T.ll = L + (x1 ? e1 : 0u) + (x2 ? e2 : 0u);
    T.lit = qq + 1u + x1 + x2;
    const uint32_t mp = T.lit + T.ll;
    const uint32_t mi = mp + mis;
    const uint32_t w1 = cin32m<kMir>(cin, mi);
    T.off = w1 & 0xFFFFu;
    const uint32_t f1 = (w1 >> 16) & 0xFFu, f2 = w1 >> 24;
    const uint32_t y1 = M == 15u ? 1u : 0u, y2 = (M == 15u && f1 == 255u) ? 1u : 0u;
    T.ml = M + 4u + (y1 ? f1 : 0u) + (y2 ? f2 : 0u);
    T.nxt = mp + 2u + y1 + y2;
    // precedence (lowest first): long match run, ext byte past the end, offset past the
    // staged input, offset cut off, last sequence, bad literal run
    uint32_t fm = (y2 && f2 == 255u) ? F_LONG : 0u;
    fm = (T.nxt > C) ? F_ERR : fm;
    fm = (mi + 4 > fill) ? F_MORE : fm;
    fm = (C - mp < 2) ? F_ERR : fm;
    fm = (mp == C) ? (mi > fill ? F_MORE : F_LAST) : fm;
    fm = (qq >= C || T.lit > C || T.ll > C - T.lit) ? F_ERR : fm;
    T.flags = fm | ((x2 && e2 == 255u) ? F_LONG : 0u);
    return T;
}

// Next-token step of a token assumed at block position qq, for the chain walk of the window at
// q: nxt - q (1..kPos-1) when the next token lies inside the window and this token is an
// ordinary sequence; kPos when the chain leaves the window here (next token at or past q + kPos,
// last sequence, malformed, long length run, or bytes past the staged input — dec_spec then
// tells which). Consistent with dec_spec: a step < kPos implies dec_spec flags are clear.
template <bool kMir = false>
__device__ __forceinline__ uint32_t dec_step(const uint8_t* cin, uint32_t qq, uint32_t q, uint32_t mis, uint32_t C,
                                             uint32_t fill) {
    using namespace dec;
    const uint32_t w0 = cin32m<kMir>(cin, qq + mis);
    const uint32_t t = w0 & 0xFFu, L = t >> 4, M = t & 15u;
    const uint32_t e1 = (w0 >> 8) & 0xFFu, e2 = (w0 >> 16) & 0xFFu;
    const bool x1 = L == 15u, x2 = x1 && e1 == 255u;
    const uint32_t mp = qq + 1u + L + (x1 ? 1u + e1 : 0u) + (x2 ? 1u + e2 : 0u);
    const uint32_t w1 = cin32m<kMir>(cin, mp + mis);
    const uint32_t f1 = (w1 >> 16) & 0xFFu, f2 = w1 >> 24;
    const bool y1 = M == 15u, y2 = y1 && f1 == 255u;
    const uint32_t nxt = mp + 2u + (y1 ? 1u : 0u) + (y2 ? 1u : 0u);
    const bool stop = (x2 && e2 == 255u) | (y2 && f2 == 255u) | (mp + mis + 4u > fill) | (nxt >= C) | (nxt - q >= kPos);
    return stop ? kPos : nxt - q;
}

// Decode one compressed block of C bytes. hist = bytes of earlier unit output matches may use.
// Output overflowing `limit` is corruption (lz4_flex: output sink bounded by the block size);
// overflowing only `cap` is DST_TOO_SMALL.
__device__ int dec_block(DecWave& w, const uint8_t* in, uint32_t C, uint32_t limit, uint32_t cap, uint32_t hist) {
    using namespace dec;
    const int lane = w.lane;
    const uint32_t bstart = w.upos;
    if (C == 0) return S3HC_CORRUPT;
    // Input ring: aligned dwords of the block (any alignment), one 256-byte chunk per lane-dword,
    // kept kAhead bytes ahead of the parse; the next chunk's load is always in flight.
    const uint32_t mis = (uint32_t)((uintptr_t)in & 3);
    const uint32_t* aw = (const uint32_t*)((uintptr_t)in - mis);
    const uint32_t kmax = (mis + C - 1) >> 2;  // last dword holding block bytes
    const uint32_t fill_end = (mis + C + kChunk - 1) & ~(kChunk - 1);
    uint32_t* cr = (uint32_t*)w.cin;
    uint32_t fill;
    uint32_t pf;
    {
        uint32_t d[kInit];
#pragma unroll
        for (uint32_t c = 0; c < kInit; ++c) {
            const uint32_t k = 64u * c + (uint32_t)lane;
            d[c] = aw[k < kmax ? k : kmax];
        }
        const uint32_t kp = 64u * kInit + (uint32_t)lane;
        pf = aw[kp < kmax ? kp : kmax];
#pragma unroll
        for (uint32_t c = 0; c < kInit; ++c) cr[64u * c + (uint32_t)lane] = d[c];
        fill = kInit * kChunk;
    }
    uint32_t q = 0;
    for (;;) {
        if (q >= C) return S3HC_CORRUPT;  // a token was expected
        {
            const uint32_t want = q + mis + kAhead < fill_end ? q + mis + kAhead : fill_end;
            if (fill < want) {
                const uint64_t t0 = PROF_NOW();
                do {
                    cr[((fill >> 2) + lane) & (kCring / 4 - 1)] = pf;
                    fill += kChunk;
                    const uint32_t kn = (fill >> 2) + lane;
                    pf = aw[kn < kmax ? kn : kmax];
                } while (fill < want);
                PROF_ADD(w.pr, 0, PROF_NOW() - t0);
                PROF_ADD(w.pr, 9, 1);
            }
            wave_sync();
        }
        const uint64_t tp0 = PROF_NOW();
        // ---- chain walk over the window's kPos token positions. Each lane evaluates the
        // next-token step at positions q + lane + 64k (k = 0..3); the scalar walk follows the true
        // chain from q (one readlane per hop) and marks members in four 64-bit masks; members are
        // then compacted into member order (mbcnt ranks through a small LDS slot table).
        const uint32_t nx0 = dec_step(w.cin, q + lane, q, mis, C, fill);
#ifdef S3HC_PROF
        uint64_t tsA = PROF_NOW();
#endif
        const uint32_t nx1 = dec_step(w.cin, q + 64 + lane, q, mis, C, fill);
        const uint32_t nx2 = dec_step(w.cin, q + 128 + lane, q, mis, C, fill);
        const uint32_t nx3 = dec_step(w.cin, q + 192 + lane, q, mis, C, fill);
#if S3HC_DEC_PK == 5
        const uint32_t nx4 = dec_step(w.cin, q + 256 + lane, q, mis, C, fill);
        uint64_t m4 = 0;
#endif
        uint64_t m0 = 0, m1 = 0, m2 = 0, m3 = 0;
        uint32_t l = 0, lastl = 0;
#ifdef S3HC_PROF
        // steps are consumed by the walk: force them complete before the walk timer starts
        __builtin_amdgcn_s_waitcnt(0);
        { const uint64_t tn = PROF_NOW(); PROF_ADD(w.pr, 12, tn - tsA); tsA = tn; }
#endif
        WALK_PRIO_ON();
        while (l < 64u) { lastl = l; m0 |= 1ull << l; l = rdl(nx0, l); }
        while (l < 128u) { lastl = l; m1 |= 1ull << (l - 64u); l = rdl(nx1, l - 64u); }
        while (l < 192u) { lastl = l; m2 |= 1ull << (l - 128u); l = rdl(nx2, l - 128u); }
        while (l < 256u) { lastl = l; m3 |= 1ull << (l - 192u); l = rdl(nx3, l - 192u); }
#if S3HC_DEC_PK == 5
        while (l < 320u) { lastl = l; m4 |= 1ull << (l - 256u); l = rdl(nx4, l - 256u); }
#endif
        WALK_PRIO_OFF();
#ifdef S3HC_PROF
        PROF_ADD(w.pr, 13, PROF_NOW() - tsA);
#endif
        // members are >= 3 bytes apart except the last, so at most kPos / 3 + 1 of them (< kMaxMem)
        const uint32_t c1 = (uint32_t)__builtin_popcountll(m0), c2 = c1 + (uint32_t)__builtin_popcountll(m1);
        const uint32_t c3 = c2 + (uint32_t)__builtin_popcountll(m2);
        uint32_t n = c3 + (uint32_t)__builtin_popcountll(m3);
#if S3HC_DEC_PK == 5
        const uint32_t c4 = n;
        n += (uint32_t)__builtin_popcountll(m4);
#endif
        {
            uint16_t* slots = w.refs;  // refs are free between passes
            auto put = [&](uint64_t m, uint32_t base, uint32_t k) {
                const uint32_t rank = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
                *(((m >> lane) & 1ull) ? slots + rank : (uint16_t*)w.sink + (lane & 31)) = (uint16_t)(64u * k + (uint32_t)lane);
            };
            put(m0, 0, 0);
            if (m1) put(m1, c1, 1);
            if (m2) put(m2, c2, 2);
            if (m3) put(m3, c3, 3);
#if S3HC_DEC_PK == 5
            if (m4) put(m4, c4, 4);
#endif
            wave_sync();
        }
        const uint32_t rp0 = w.refs[lane];
        const uint32_t rp1 = n > 64u ? w.refs[64 + lane] : 0u;
        // ---- members decoded densely: member m's token in lane m (set 0) / m - 64 (set 1)
        const DecTok t0 = dec_spec(w.cin, q + rp0, mis, C, fill);
        DecTok t1 = {0u, 0u, 0u, 0u, 0u, 0u};
        if (n > 64u) t1 = dec_spec(w.cin, q + rp1, mis, C, fill);
        auto rd2 = [&](uint32_t v0, uint32_t v1, uint32_t m) -> uint32_t { return m < 64 ? rdl(v0, m) : rdl(v1, m - 64); };
        int stop = 0;  // 0 window exhausted, 1 last sequence, 2 error, 3 slow path at cur, 4 long sequence
        uint32_t cur, cm = 0;  // cm: member run by the long-sequence path (stop 4)
        {
            const uint32_t fl = rd2(t0.flags, t1.flags, n - 1u);
            if (fl & (F_LONG | F_MORE | F_ERR)) {
                --n;  // the chain's last token goes to the slow path (or is an error)
                stop = (fl & (F_LONG | F_MORE)) ? 3 : 2;
                cur = q + lastl;
            } else if (fl & F_LAST) {
                stop = 1;
                cur = C;
            } else {
                cur = rd2(t0.nxt, t1.nxt, n - 1u);
            }
        }
        const uint64_t tp1 = PROF_NOW();
        PROF_ADD(w.pr, 1, tp1 - tp0);
        if (n) {
            bool isM0 = (uint32_t)lane < n, isM1 = (uint32_t)lane + 64u < n;
            const uint32_t sl0 = isM0 ? t0.ll + ((t0.flags & F_LAST) ? 0u : t0.ml) : 0u;
            const uint32_t sl1 = isM1 ? t1.ll + ((t1.flags & F_LAST) ? 0u : t1.ml) : 0u;
            const uint32_t orel0 = wave_excl_scan(sl0, lane);
            const uint32_t tot0 = rdl(orel0 + sl0, 63);
            uint32_t orel1 = tot0;
            uint32_t S = tot0;
            if (n > 64u) {
                orel1 = tot0 + wave_excl_scan(sl1, lane);
                S = rdl(orel1 + sl1, 63);
            }
            // output budget: the members that fit in kWin run now, the rest next window
            const uint64_t cut0 = __ballot(isM0 && orel0 + sl0 > kWin);
            const uint64_t cut1 = __ballot(isM1 && orel1 + sl1 > kWin);
            if (cut0 | cut1) {
                const uint32_t c = cut0 ? (uint32_t)__builtin_ctzll(cut0) : 64u + (uint32_t)__builtin_ctzll(cut1);
                n = c;
                isM0 = (uint32_t)lane < n;
                isM1 = (uint32_t)lane + 64u < n;
                S = rd2(orel0, orel1, c);
                stop = n ? 0 : 4;
                cm = c;
                cur = q + rd2(rp0, rp1, c);
            }
            if (n) {
                // lz4_flex bound checks, lane-parallel; the first failing member decides
                const uint32_t base = w.upos - bstart;
                auto check = [&](const DecTok& T, uint32_t orel) -> int {
                    const uint32_t produced = base + orel;
                    const bool lastm = (T.flags & F_LAST) != 0;
                    const uint32_t have = produced + T.ll;
                    int st = S3HC_OK;
                    st = (!lastm && T.ml > cap - have) ? S3HC_DST_TOO_SMALL : st;
                    st = (!lastm && T.ml > limit - have) ? S3HC_CORRUPT : st;
                    st = (!lastm && (T.off == 0 || T.off > have + hist)) ? S3HC_CORRUPT : st;
                    st = (T.ll > cap - produced) ? S3HC_DST_TOO_SMALL : st;
                    st = (T.ll > limit - produced) ? S3HC_CORRUPT : st;
                    return st;
                };
                const int st0 = check(t0, orel0), st1 = check(t1, orel1);
                const uint64_t bad0 = __ballot(isM0 && st0 != S3HC_OK);
                const uint64_t bad1 = __ballot(isM1 && st1 != S3HC_OK);
                if (bad0) return (int)rdl((uint32_t)st0, (uint32_t)__builtin_ctzll(bad0));
                if (bad1) return (int)rdl((uint32_t)st1, (uint32_t)__builtin_ctzll(bad1));
                dec_window_exec(w, S, isM0, isM1, orel0, orel1, sl0, sl1, t0.ll, t1.ll, t0.off, t1.off,
                                (t0.lit + mis) & kCmask, (t1.lit + mis) & kCmask);
                PROF_ADD(w.pr, 2, PROF_NOW() - tp1);
                PROF_ADD(w.pr, 5, 1);
                PROF_ADD(w.pr, 6, n);
                PROF_ADD(w.pr, 7, (S + 255) / 256);
                PROF_ADD(w.pr, 11, S);
            }
        }
        const uint64_t tp2 = PROF_NOW();
        if (stop == 1) return S3HC_OK;
        if (stop == 2) return S3HC_CORRUPT;
        if (stop == 4) {
            const uint32_t c = cm;
            const uint32_t f = rd2(t0.flags, t1.flags, c);
            const int rc = dec_seq(w, in, rd2(t0.lit, t1.lit, c), rd2(t0.ll, t1.ll, c), (f & F_LAST) != 0,
                                   rd2(t0.off, t1.off, c), rd2(t0.ml, t1.ml, c), mis, fill, bstart, limit, cap, hist);
            if (rc) return rc;
            if (f & F_LAST) return S3HC_OK;
            cur = rd2(t0.nxt, t1.nxt, c);
        }
        if (stop == 3) {
            // Slow path: this sequence has long length runs or reaches past the stage.
            uint32_t pos = cur;
            const uint32_t t = in[pos];
            pos++;
            uint32_t sll = t >> 4;
            if (sll == 15 && dec_ext_scan(in, C, pos, sll, lane)) return S3HC_CORRUPT;
            if (sll > C - pos) return S3HC_CORRUPT;
            const uint32_t slit = pos;
            pos += sll;
            if (pos == C) return dec_seq(w, in, slit, sll, true, 0, 0, mis, fill, bstart, limit, cap, hist);
            const uint32_t produced = w.upos - bstart;
            if (sll > limit - produced) return S3HC_CORRUPT;
            if (sll > cap - produced) return S3HC_DST_TOO_SMALL;
            if (C - pos < 2) return S3HC_CORRUPT;
            const uint32_t soff = (uint32_t)in[pos] | ((uint32_t)in[pos + 1] << 8);
            pos += 2;
            uint32_t sml = (t & 15) + 4;
            if ((t & 15) == 15 && dec_ext_scan(in, C, pos, sml, lane)) return S3HC_CORRUPT;
            const int rc = dec_seq(w, in, slit, sll, false, soff, sml, mis, fill, bstart, limit, cap, hist);
            if (rc) return rc;
            cur = pos;
        }
        PROF_ADD(w.pr, 3, PROF_NOW() - tp2);
        q = cur;
    }
}

// units [0, count) of a plan: count read on the device (a device-built plan: the frame walk's
// block total) or the launch's cap; grids stride over them
__device__ __forceinline__ uint32_t unit_count(const uint64_t* ucount, uint32_t cap) {
    return ucount ? (uint32_t)min<uint64_t>(*ucount, (uint64_t)cap) : cap;
}

#ifndef S3HC_DEC_LDS_PAD
#define S3HC_DEC_LDS_PAD 0  // diagnostic builds: extra LDS per workgroup to lower occupancy
#endif
// The one-wave-per-unit decoder (round 1's default; S3HC_DEC_ONEWAVE=1) is a comparison variant:
// compiled only into diagnostic builds (make diag DIAG=-DS3HC_DIAG_VARIANTS=1), never shipped.
#if S3HC_DIAG_VARIANTS
__device__ __forceinline__ void decode_unit_wave(const uint32_t u, uint8_t* smem, const uint8_t* __restrict__ src,
                                                 uint8_t* dst, const DecBlock* __restrict__ blk,
                                                 const DecUnit* __restrict__ units, uint32_t* __restrict__ blk_out,
                                                 int32_t* __restrict__ blk_status, const uint8_t* __restrict__ unit_lb,
                                                 const uint8_t* __restrict__ unit_fast) {
    const int lane = lane_id();
    const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    if (unit_lb && unit_lb[u]) return;  // decoded by the large-block path (s3hc_lb.hip)
    if (unit_fast && unit_fast[u]) return;  // decoded by the 64 KiB-block path (s3hc_fast.hip)
    const DecUnit U = units[u];
    if (U.n == 0) return;
    DecWave w;
    w.ring = smem + wv * dec::kWaveLds;
    w.cin = w.ring + dec::kRing;
    w.marks = w.cin + dec::kCring;
    w.refs = (uint16_t*)(w.marks + dec::kMarks);
    w.sink = (uint8_t*)(w.refs + dec::kRefs);
    w.mtab = (uint2*)(w.sink + dec::kSink);
    w.mmax = dec::kMaxMem - 1;
    for (uint32_t i = (uint32_t)lane; i < dec::kMarks / 16; i += 64) ((uint4*)w.marks)[i] = make_uint4(0, 0, 0, 0);
    w.out = dst + blk[U.first].dst_off;
    w.upos = 0;
    w.flushed = 0;
    w.lane = lane;
    int status = S3HC_OK;
#ifdef S3HC_PROF
    for (int k = 0; k < 16; ++k) w.pr[k] = 0;
    const uint64_t tk0 = PROF_NOW();
#endif
    for (uint32_t b = 0; b < U.n; ++b) {
        const DecBlock B = blk[U.first + b];
        const uint32_t start = w.upos;
        if (status == S3HC_OK) {
            const uint8_t* in = src + B.src_off;
            const uint32_t hist = (B.flags & DB_LINKED) ? start : 0u;
            if (B.flags & DB_STORED) {
                if (B.csize > B.limit) status = S3HC_CORRUPT;
                else if (B.csize > B.cap) status = S3HC_DST_TOO_SMALL;
                else if (U.n == 1) {
                    wave_copy_global(w.out, in, B.csize, lane);
                    w.upos = w.flushed = B.csize;
                } else {
                    dec_literals(w, in, 0, B.csize, 0xFFFFFFFFu, false);
                }
            } else {
                status = dec_block(w, in, B.csize, B.limit, B.cap, hist);
            }
        }
        if (lane == 0) {
            blk_out[U.first + b] = status == S3HC_OK ? w.upos - start : 0u;
            blk_status[U.first + b] = status;
        }
    }
    dec_final_flush(w);
#ifdef S3HC_PROF
    w.pr[4] = PROF_NOW() - tk0;
    if (lane == 0)
        for (int k = 0; k < 16; ++k) atomicAdd(&g_prof[k], (unsigned long long)w.pr[k]);
#endif
}

__global__ __launch_bounds__(256) void k_decode_units(const uint8_t* __restrict__ src, uint8_t* dst,
                                                      const DecBlock* __restrict__ blk,
                                                      const DecUnit* __restrict__ units, uint32_t nunits,
                                                      const uint64_t* __restrict__ ucount,
                                                      uint32_t* __restrict__ blk_out,
                                                      int32_t* __restrict__ blk_status,
                                                      const uint8_t* __restrict__ unit_lb,
                                                      const uint8_t* __restrict__ unit_fast) {
    __shared__ __attribute__((aligned(16))) uint8_t smem[dec::kWaves * dec::kWaveLds + S3HC_DEC_LDS_PAD];
    const uint32_t nu = unit_count(ucount, nunits);
    const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    for (uint32_t ub = blockIdx.x; ub * dec::kWaves < nu; ub += gridDim.x) {  // (each wave on its own LDS)
        const uint32_t u = ub * dec::kWaves + wv;
        if (u < nu) decode_unit_wave(u, smem, src, dst, blk, units, blk_out, blk_status, unit_lb, unit_fast);
    }
}
#endif  // S3HC_DIAG_VARIANTS

// ====================================================== decode, parser + executor waves
// k_decode_pe: the same decoder with the two halves of a window on two waves of one 128-thread
// workgroup per unit. Wave P walks the token chain (staging, next-token steps, the serial
// readlane walk, member decode, lz4_flex bound checks) and writes one command per step into a
// two-slot LDS queue; wave E executes the command P wrote one step earlier (marks, the
// byte-parallel passes, long sequences, stored blocks, flushes). Both waves meet at one
// workgroup barrier per step, so a step costs max(parse, execute) instead of their sum, and a
// 4096-block batch runs 8 waves per SIMD instead of 4 (10 KiB of LDS and <= 64 VGPRs a unit).
// Statuses and output sizes are written by P (lane 0), the output bytes by E.
namespace dpe {
constexpr uint32_t kMaxMem = 88;  // members of one window: at most kPos / 3 + 1 = 86
enum : uint32_t { C_NOP = 0, C_WIN = 1, C_STORED = 2, C_END = 3 };
struct Slot {
    uint32_t cmd;
    uint32_t S;       // WIN: output bytes of the members
    uint32_t n;       // WIN: members
    uint32_t far;     // WIN: a member reads a source older than the output ring
    uint64_t ptr;     // WIN tail / STORED: compressed block base in HBM
    uint32_t tail;    // WIN: 0 none, 1 one sequence follows the members, 2 it is the block's last
    uint32_t tlit;    // tail literal start (block offset) / STORED: size
    uint32_t tll, toff, tml;
    uint32_t single;  // STORED: the unit's only block (copied straight to HBM)
    uint2 mtab[kMaxMem];
    uint16_t orel[kMaxMem];  // member's first window byte; 0xFFFF = produces nothing
};
constexpr uint32_t kSlot = (uint32_t)((sizeof(Slot) + 15) & ~(size_t)15);
constexpr uint32_t kPslots = 256;  // P: member compaction table (u16 per member, 128 entries)
constexpr uint32_t kMirror = 16;  // the input ring is followed by a copy of its first dword
constexpr uint32_t kLds = dec::kRing + dec::kCring + kMirror + dec::kMarks + 2 * dec::kRefs + dec::kSink + 2 * kSlot + kPslots + 16;
static_assert(kLds <= 10240, "16 units per CU (a 4096-block batch resident at once) need <= 10 KiB each");
}  // namespace dpe

#ifndef S3HC_PE_WAVES_PER_EU
#define S3HC_PE_WAVES_PER_EU 8
#endif
__device__ __forceinline__ void decode_unit_pe(
    const uint32_t u, uint8_t* smem, const uint8_t* __restrict__ src, uint8_t* dst, const DecBlock* __restrict__ blk,
    const DecUnit* __restrict__ units, uint32_t* __restrict__ blk_out, int32_t* __restrict__ blk_status,
    const uint8_t* __restrict__ unit_lb, const uint8_t* __restrict__ unit_fast) {
    using namespace dec;
    using dpe::Slot;
    if (unit_lb && unit_lb[u]) return;  // decoded by the large-block path (s3hc_lb.hip)
    if (unit_fast && unit_fast[u]) return;  // decoded by the 64 KiB-block path (s3hc_fast.hip)
    const DecUnit U = units[u];
    if (U.n == 0) return;
    const int lane = lane_id();
    const bool isP = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) == 0;
    uint8_t* ring = smem;
    uint8_t* cin = ring + kRing;
    uint8_t* marks = cin + kCring + dpe::kMirror;
    uint16_t* refs = (uint16_t*)(marks + kMarks);
    uint8_t* sink = (uint8_t*)(refs + kRefs);
    Slot* slots = (Slot*)(sink + kSink);
    uint16_t* pslots = (uint16_t*)((uint8_t*)slots + 2 * dpe::kSlot);
    volatile uint32_t* done = (volatile uint32_t*)((uint8_t*)pslots + dpe::kPslots);

    // ---- E state
    DecWave w;
    w.ring = ring;
    w.cin = cin;
    w.marks = marks;
    w.refs = refs;
    w.sink = sink;
    w.mtab = slots[0].mtab;
    w.mmax = dpe::kMaxMem - 1;
    w.out = dst + blk[U.first].dst_off;
    w.upos = 0;
    w.flushed = 0;
    w.lane = lane;
    // ---- P state (wave-uniform except pf)
    uint32_t b = 0;          // next block of the unit
    int status = S3HC_OK;
    uint32_t upos = 0;       // unit bytes produced by everything emitted so far
    uint32_t bstart = 0;     // upos at the start of the current block
    bool inblk = false;      // inside a compressed block
    bool ended = false;
    uint32_t prev_lo = 0xFFFFFFFFu;  // input-ring start of the window E executes this step (none)
    const uint8_t* in = nullptr;
    const uint32_t* aw = nullptr;
    uint32_t C = 0, limit = 0, cap = 0, hist = 0, mis = 0, kmax = 0, fill_end = 0, fill = 0, q = 0, pf = 0;
    if (!isP) {
        for (uint32_t i = (uint32_t)lane; i < kMarks / 16; i += 64) ((uint4*)marks)[i] = make_uint4(0, 0, 0, 0);
        if (lane == 0) *done = 0u;
    }
    for (uint32_t it = 0;; ++it) {
        if (isP) {
            Slot& sl = slots[it & 1u];
            uint32_t cmd = dpe::C_NOP;
            uint32_t emit_lo = 0xFFFFFFFFu;
            // block bookkeeping: P knows every block's size and status before E has run it
            auto finish_block = [&](int st) {
                if (lane == 0) {
                    blk_out[U.first + b] = st == S3HC_OK ? upos - bstart : 0u;
                    blk_status[U.first + b] = st;
                }
                status = st;
                inblk = false;
                ++b;
            };
            while (!ended && cmd == dpe::C_NOP) {
                if (!inblk) {
                    if (b == U.n) {
                        cmd = dpe::C_END;
                        ended = true;
                        break;
                    }
                    const DecBlock B = blk[U.first + b];
                    bstart = upos;
                    if (status != S3HC_OK) {
                        finish_block(status);
                        continue;
                    }
                    in = src + B.src_off;
                    if (B.flags & DB_STORED) {
                        if (B.csize > B.limit) { finish_block(S3HC_CORRUPT); continue; }
                        if (B.csize > B.cap) { finish_block(S3HC_DST_TOO_SMALL); continue; }
                        cmd = dpe::C_STORED;
                        if (lane == 0) {
                            sl.ptr = (uint64_t)(uintptr_t)in;
                            sl.tlit = B.csize;
                            sl.single = U.n == 1 ? 1u : 0u;
                        }
                        upos += B.csize;
                        finish_block(S3HC_OK);
                        break;
                    }
                    if (B.csize == 0) { finish_block(S3HC_CORRUPT); continue; }
                    if (prev_lo != 0xFFFFFFFFu) break;  // E still reads the input ring: restage next step
                    C = B.csize;
                    limit = B.limit;
                    cap = B.cap;
                    hist = (B.flags & DB_LINKED) ? upos : 0u;
                    mis = (uint32_t)((uintptr_t)in & 3);
                    aw = (const uint32_t*)((uintptr_t)in - mis);
                    kmax = (mis + C - 1) >> 2;
                    fill_end = (mis + C + kChunk - 1) & ~(kChunk - 1);
                    {
                        uint32_t d[kInit];
#pragma unroll
                        for (uint32_t c = 0; c < kInit; ++c) {
                            const uint32_t k = 64u * c + (uint32_t)lane;
                            d[c] = aw[k < kmax ? k : kmax];
                        }
                        const uint32_t kp = 64u * kInit + (uint32_t)lane;
                        pf = aw[kp < kmax ? kp : kmax];
#pragma unroll
                        for (uint32_t c = 0; c < kInit; ++c) ((uint32_t*)cin)[64u * c + (uint32_t)lane] = d[c];
                        if (lane == 0) ((uint32_t*)cin)[kCring / 4] = d[0];  // mirror of the ring's first dword
                        fill = kInit * kChunk;
                    }
                    q = 0;
                    inblk = true;
                }
                // ---- one window at q
                if (q >= C) { finish_block(S3HC_CORRUPT); continue; }
                {
                    const uint32_t want = q + mis + kAhead < fill_end ? q + mis + kAhead : fill_end;
                    // the window E executes this step reads input-ring bytes from prev_lo on
                    const uint32_t guard = prev_lo == 0xFFFFFFFFu ? 0xFFFFFFFFu : prev_lo + kCring - kChunk;
                    while (fill < want && fill <= guard) {
                        const uint32_t ci = ((fill >> 2) + lane) & (kCring / 4 - 1);
                        ((uint32_t*)cin)[ci] = pf;
                        if (ci == 0) ((uint32_t*)cin)[kCring / 4] = pf;  // mirror
                        fill += kChunk;
                        const uint32_t kn = (fill >> 2) + (uint32_t)lane;
                        pf = aw[kn < kmax ? kn : kmax];
                    }
                    wave_sync();
                }
                const uint32_t nx0 = dec_step<true>(cin, q + lane, q, mis, C, fill);
                const uint32_t nx1 = dec_step<true>(cin, q + 64 + lane, q, mis, C, fill);
                const uint32_t nx2 = dec_step<true>(cin, q + 128 + lane, q, mis, C, fill);
                const uint32_t nx3 = dec_step<true>(cin, q + 192 + lane, q, mis, C, fill);
                uint64_t m0 = 0, m1 = 0, m2 = 0, m3 = 0;
                uint32_t l = 0, lastl = 0;
                WALK_PRIO_ON();
                while (l < 64u) { lastl = l; m0 |= 1ull << l; l = rdl(nx0, l); }
                while (l < 128u) { lastl = l; m1 |= 1ull << (l - 64u); l = rdl(nx1, l - 64u); }
                while (l < 192u) { lastl = l; m2 |= 1ull << (l - 128u); l = rdl(nx2, l - 128u); }
                while (l < 256u) { lastl = l; m3 |= 1ull << (l - 192u); l = rdl(nx3, l - 192u); }
                WALK_PRIO_OFF();
                const uint32_t c1 = (uint32_t)__builtin_popcountll(m0), c2 = c1 + (uint32_t)__builtin_popcountll(m1);
                const uint32_t c3 = c2 + (uint32_t)__builtin_popcountll(m2);
                uint32_t n = c3 + (uint32_t)__builtin_popcountll(m3);
                {
                    auto put = [&](uint64_t m, uint32_t base, uint32_t k) {
                        const uint32_t rank = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
                        *(((m >> lane) & 1ull) ? pslots + rank : (uint16_t*)sink + (lane & 31)) = (uint16_t)(64u * k + (uint32_t)lane);
                    };
                    put(m0, 0, 0);
                    if (m1) put(m1, c1, 1);
                    if (m2) put(m2, c2, 2);
                    if (m3) put(m3, c3, 3);
                    wave_sync();
                }
                const uint32_t rp0 = pslots[lane];
                const uint32_t rp1 = n > 64u ? pslots[64 + lane] : 0u;
                const DecTok t0 = dec_spec<true>(cin, q + rp0, mis, C, fill);
                DecTok t1 = {0u, 0u, 0u, 0u, 0u, 0u};
                if (n > 64u) t1 = dec_spec<true>(cin, q + rp1, mis, C, fill);
                auto rd2 = [&](uint32_t v0, uint32_t v1, uint32_t m) -> uint32_t { return m < 64 ? rdl(v0, m) : rdl(v1, m - 64); };
                int stop = 0;  // 0 window exhausted, 1 last sequence, 2 error, 3 slow path at cur, 4 long sequence
                uint32_t cur, cm = 0;
                {
                    const uint32_t fl = rd2(t0.flags, t1.flags, n - 1u);
                    if (fl & (F_LONG | F_MORE | F_ERR)) {
                        --n;
                        stop = (fl & (F_LONG | F_MORE)) ? 3 : 2;
                        cur = q + lastl;
                    } else if (fl & F_LAST) {
                        stop = 1;
                        cur = C;
                    } else {
                        cur = rd2(t0.nxt, t1.nxt, n - 1u);
                    }
                }
                uint32_t S = 0;
                if (n) {
                    bool isM0 = (uint32_t)lane < n, isM1 = (uint32_t)lane + 64u < n;
                    const uint32_t sl0 = isM0 ? t0.ll + ((t0.flags & F_LAST) ? 0u : t0.ml) : 0u;
                    const uint32_t sl1 = isM1 ? t1.ll + ((t1.flags & F_LAST) ? 0u : t1.ml) : 0u;
                    const uint32_t orel0 = wave_excl_scan(sl0, lane);
                    const uint32_t tot0 = rdl(orel0 + sl0, 63);
                    uint32_t orel1 = tot0;
                    S = tot0;
                    if (n > 64u) {
                        orel1 = tot0 + wave_excl_scan(sl1, lane);
                        S = rdl(orel1 + sl1, 63);
                    }
                    const uint64_t cut0 = __ballot(isM0 && orel0 + sl0 > kWin);
                    const uint64_t cut1 = __ballot(isM1 && orel1 + sl1 > kWin);
                    if (cut0 | cut1) {
                        const uint32_t c = cut0 ? (uint32_t)__builtin_ctzll(cut0) : 64u + (uint32_t)__builtin_ctzll(cut1);
                        n = c;
                        isM0 = (uint32_t)lane < n;
                        isM1 = (uint32_t)lane + 64u < n;
                        S = rd2(orel0, orel1, c);
                        stop = n ? 0 : 4;
                        cm = c;
                        cur = q + rd2(rp0, rp1, c);
                    }
                    if (n) {
                        const uint32_t base = upos - bstart;
                        auto check = [&](const DecTok& T, uint32_t orel) -> int {
                            const uint32_t produced = base + orel;
                            const bool lastm = (T.flags & F_LAST) != 0;
                            const uint32_t have = produced + T.ll;
                            int st = S3HC_OK;
                            st = (!lastm && T.ml > cap - have) ? S3HC_DST_TOO_SMALL : st;
                            st = (!lastm && T.ml > limit - have) ? S3HC_CORRUPT : st;
                            st = (!lastm && (T.off == 0 || T.off > have + hist)) ? S3HC_CORRUPT : st;
                            st = (T.ll > cap - produced) ? S3HC_DST_TOO_SMALL : st;
                            st = (T.ll > limit - produced) ? S3HC_CORRUPT : st;
                            return st;
                        };
                        const int st0 = check(t0, orel0);
                        const int st1 = n > 64u ? check(t1, orel1) : S3HC_OK;
                        const uint64_t bad0 = __ballot(isM0 && st0 != S3HC_OK);
                        const uint64_t bad1 = n > 64u ? __ballot(isM1 && st1 != S3HC_OK) : 0ull;
                        if (bad0 | bad1) {
                            finish_block(bad0 ? (int)rdl((uint32_t)st0, (uint32_t)__builtin_ctzll(bad0))
                                              : (int)rdl((uint32_t)st1, (uint32_t)__builtin_ctzll(bad1)));
                            continue;
                        }
                        // member table: (M | E << 16, L | off << 16) as dec_window_exec builds it
                        auto entry = [](uint32_t orel, uint32_t ll, uint32_t off, uint32_t lr) -> uint2 {
                            const uint32_t M = orel + ll;
                            const uint32_t E = M + off < 0xFFFFu ? M + off : 0xFFFFu;
                            return make_uint2(M | (E << 16), ((lr - orel) & 0xFFFFu) | (off << 16));
                        };
                        if (isM0) {
                            sl.mtab[lane] = entry(orel0, t0.ll, t0.off, (t0.lit + mis) & kCmask);
                            sl.orel[lane] = sl0 ? (uint16_t)orel0 : (uint16_t)0xFFFFu;
                        }
                        if (isM1) {
                            sl.mtab[64 + lane] = entry(orel1, t1.ll, t1.off, (t1.lit + mis) & kCmask);
                            sl.orel[64 + lane] = sl1 ? (uint16_t)orel1 : (uint16_t)0xFFFFu;
                        }
                        const uint32_t wu = upos;  // E's output position at this window
                        const bool far = (wu > kRing - S) &&
                                         __ballot((isM0 && sl0 > t0.ll && t0.off > kRing - S) ||
                                                  (isM1 && sl1 > t1.ll && t1.off > kRing - S));
                        if (lane == 0) sl.far = far ? 1u : 0u;
                        upos += S;
                    }
                }
                // the window's trailing single sequence (too long for a window, or past the staged input)
                uint32_t tail = 0, tlit = 0, tll = 0, toff = 0, tml = 0;
                bool blk_done = stop == 1;
                if (stop == 2) { finish_block(S3HC_CORRUPT); continue; }
                if (stop == 4) {
                    const uint32_t c = cm;
                    const uint32_t f = rd2(t0.flags, t1.flags, c);
                    tlit = rd2(t0.lit, t1.lit, c);
                    tll = rd2(t0.ll, t1.ll, c);
                    toff = rd2(t0.off, t1.off, c);
                    tml = rd2(t0.ml, t1.ml, c);
                    tail = (f & F_LAST) ? 2u : 1u;
                    if (!(f & F_LAST)) cur = rd2(t0.nxt, t1.nxt, c);
                } else if (stop == 3) {
                    uint32_t pos = cur;
                    const uint32_t t = in[pos];
                    pos++;
                    uint32_t sll = t >> 4;
                    if (sll == 15 && dec_ext_scan(in, C, pos, sll, lane)) { finish_block(S3HC_CORRUPT); continue; }
                    if (sll > C - pos) { finish_block(S3HC_CORRUPT); continue; }
                    tlit = pos;
                    tll = sll;
                    pos += sll;
                    if (pos == C) {
                        tail = 2;
                    } else {
                        if (C - pos < 2) { finish_block(S3HC_CORRUPT); continue; }
                        toff = (uint32_t)in[pos] | ((uint32_t)in[pos + 1] << 8);
                        pos += 2;
                        uint32_t sml = (t & 15) + 4;
                        if ((t & 15) == 15 && dec_ext_scan(in, C, pos, sml, lane)) { finish_block(S3HC_CORRUPT); continue; }
                        tml = sml;
                        tail = 1;
                        cur = pos;
                    }
                }
                if (tail) {
                    // dec_seq's checks, in stream order
                    const uint32_t produced = upos - bstart;
                    int st = S3HC_OK;
                    if (tll > limit - produced) st = S3HC_CORRUPT;
                    else if (tll > cap - produced) st = S3HC_DST_TOO_SMALL;
                    else if (tail == 1) {
                        const uint32_t have = produced + tll;
                        if (toff == 0 || toff > have + hist) st = S3HC_CORRUPT;
                        else if (tml > limit - have) st = S3HC_CORRUPT;
                        else if (tml > cap - have) st = S3HC_DST_TOO_SMALL;
                    }
                    if (st != S3HC_OK) { finish_block(st); continue; }
                    upos += tll + (tail == 1 ? tml : 0u);
                    blk_done = tail == 2;
                }
                if (n == 0 && tail == 0) {
                    // nothing to execute (a window whose only token is the block's empty last sequence)
                    if (blk_done) finish_block(S3HC_OK);
                    else q = cur;
                    continue;
                }
                cmd = dpe::C_WIN;
                emit_lo = n ? q + mis : 0xFFFFFFFFu;
                if (lane == 0) {
                    sl.S = S;
                    sl.n = n;
                    sl.ptr = (uint64_t)(uintptr_t)in;
                    sl.tail = tail;
                    sl.tlit = tlit;
                    sl.tll = tll;
                    sl.toff = toff;
                    sl.tml = tml;
                }
                if (blk_done) finish_block(S3HC_OK);
                else q = cur;
            }
            if (lane == 0) sl.cmd = cmd;
            prev_lo = emit_lo;
        } else if (it > 0) {
            const Slot& sl = slots[(it - 1u) & 1u];
            // the header is wave-uniform: scalar copies keep E's loops and branches scalar
            auto rfl = [](uint32_t v) -> uint32_t { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); };
            const uint32_t cmd = rfl(sl.cmd);
            const uint8_t* sptr = (const uint8_t*)(uintptr_t)(((uint64_t)rfl((uint32_t)(sl.ptr >> 32)) << 32) |
                                                              rfl((uint32_t)sl.ptr));
            if (cmd == dpe::C_WIN) {
                const uint32_t n = rfl(sl.n);
                if (n) {
                    const uint32_t a0 = w.upos & 3u;
                    const uint32_t r0 = (uint32_t)lane < n ? sl.orel[lane] : 0xFFFFu;
                    const uint32_t r1 = (uint32_t)lane + 64u < n ? sl.orel[64 + lane] : 0xFFFFu;
                    *(r0 != 0xFFFFu ? marks + r0 + a0 : sink + lane) = (uint8_t)(lane + 1);
                    *(r1 != 0xFFFFu ? marks + r1 + a0 : sink + lane) = (uint8_t)(lane + 65);
                    w.mtab = const_cast<uint2*>(sl.mtab);
                    wave_sync();
#ifndef S3HC_DIAG_NOEXEC  // diagnostic builds: P alone (instruction counts of the parse half)
                    dec_window_passes(w, rfl(sl.S), rfl(sl.far) != 0u);
#else
                    w.upos += rfl(sl.S);
#endif
                }
                const uint32_t tail = rfl(sl.tail);
                if (tail) {
                    dec_literals(w, sptr, rfl(sl.tlit), rfl(sl.tll), 0xFFFFFFFFu, false);
                    if (tail == 1) dec_match(w, rfl(sl.toff), rfl(sl.tml));
                }
            } else if (cmd == dpe::C_STORED) {
                const uint32_t cs = rfl(sl.tlit);
                if (rfl(sl.single)) {
                    wave_copy_global(w.out, sptr, cs, lane);
                    w.upos = w.flushed = cs;
                } else {
                    dec_literals(w, sptr, 0, cs, 0xFFFFFFFFu, false);
                }
            } else if (cmd == dpe::C_END) {
                dec_final_flush(w);
                if (lane == 0) *done = 1u;
            }
        }
        __syncthreads();
        if (*done) break;
    }
}

__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(S3HC_PE_WAVES_PER_EU, 8))) void k_decode_pe(
    const uint8_t* __restrict__ src, uint8_t* dst, const DecBlock* __restrict__ blk, const DecUnit* __restrict__ units,
    uint32_t nunits, const uint64_t* __restrict__ ucount, uint32_t* __restrict__ blk_out,
    int32_t* __restrict__ blk_status, const uint8_t* __restrict__ unit_lb, const uint8_t* __restrict__ unit_fast) {
    __shared__ __attribute__((aligned(16))) uint8_t smem[dpe::kLds];
    const uint32_t nu = unit_count(ucount, nunits);
    for (uint32_t u = blockIdx.x; u < nu; u += gridDim.x) {
        decode_unit_pe(u, smem, src, dst, blk, units, blk_out, blk_status, unit_lb, unit_fast);
        __syncthreads();  // (the next unit reuses the LDS)
    }
}

// ================================================================== encode
namespace enc {
constexpr uint32_t kPad = 16;                               // front pad: reads at i-8 stay in bounds
constexpr uint32_t kGIn = kPad + kPrewarm + kGroupSegs * kSeg + 128;  // a group's staged input (+ read-ahead)
constexpr uint32_t kGThreads = 64 * kGroupSegs;
constexpr uint32_t kTbl = 1u << kHashLog;
#ifndef S3HC_STEPS
#define S3HC_STEPS 8
#endif
#ifndef S3HC_SHORT_GATE  // distance-1..4 candidate only without a verified table one (0: also under a short one)
#define S3HC_SHORT_GATE 1
#endif
#ifndef S3HC_LAZY  // lazy match selection (diagnostic builds: 0 = plain greedy)
#define S3HC_LAZY 1
#endif
#ifndef S3HC_SALU_PAD
#define S3HC_SALU_PAD 0
#endif
#ifndef S3HC_VALU_PAD
#define S3HC_VALU_PAD 0
#endif
#ifndef S3HC_ABL  // diagnostic ablations of the match finder's phases (never shipped)
#define S3HC_ABL 0
#endif
#ifndef S3HC_ENC_MINWAVES
#define S3HC_ENC_MINWAVES 1
#endif
constexpr uint32_t kSteps = S3HC_STEPS;                     // 64-position steps per sub-block
constexpr uint32_t kStash = 64 * kSteps / 4;                // hops per sub-block (a hop covers >= 4 bytes)
// Encoder modes (s3hc_set_encode_mode): the match finder is instantiated per mode.
//   kPS  positions per lane and step: every position is inserted into the table, the first of a
//        lane's kPS is probed (a match starting at one of the others is found by the backward
//        extension of the next probe)
//   kIns positions with (P & kIns) != 0 are probed but not inserted (fewer entries overwritten:
//        a better ratio with lazy selection)
//   fast  (default): kPS 2, kIns 0;   small: kPS 1, kIns 1
#ifndef S3HC_FWD_DW
#define S3HC_FWD_DW 6
#endif
constexpr int kNQ = S3HC_FWD_DW;                            // dwords compared past the first 4 bytes
constexpr uint32_t kFwd = 3 + 4 * kNQ;                      // forward bytes measured per probe; a probe
                                                            // reaching kFwd is extended in the walk
constexpr uint32_t kEmpty = 0xFFFFu;
}  // namespace enc

// LZ4 length-extension bytes for a length field of n: (n - 15) / 255 + 1 for n >= 15, else 0
// (branch-free form: (n + 240) / 255).
__device__ __forceinline__ uint32_t ext_bytes(uint32_t n) { return (n + 240u) / 255u; }
// v_ffbl_b32 / v_ffbh_u32 with the hardware's answer for 0 (all ones), so a chain of
// first-mismatch tests is a min over saturating adds instead of compare + select per dword.
__device__ __forceinline__ uint32_t ffbl_hw(uint32_t x) {
    uint32_t r;
    asm("v_ffbl_b32 %0, %1" : "=v"(r) : "v"(x));
    return r;
}
__device__ __forceinline__ uint32_t ffbh_hw(uint32_t x) {
    uint32_t r;
    asm("v_ffbh_u32 %0, %1" : "=v"(r) : "v"(x));
    return r;
}
// Bytes equal after the first 4 of a match: first differing byte of the kNQ dword pairs
// (d[j] = XOR of dword j + 1), 4 + 4j + byte; kFwd + a lot when all are equal.
template <int N>
__device__ __forceinline__ uint32_t fwd_len(const uint32_t (&d)[N]) {
    uint32_t m = ffbl_hw(d[0]);
#pragma unroll
    for (int j = 1; j < N; ++j) m = umin32(m, __builtin_elementwise_add_sat(ffbl_hw(d[j]), 32u * (uint32_t)j));
    return (m >> 3) + 4u;
}
__device__ __forceinline__ uint32_t hash4(uint32_t v) { return (v * 2654435761u) >> (32 - kHashLog); }
// Table hash of the 4 bytes v at a position and the byte after them (b5): a 5-byte hash
__device__ __forceinline__ uint32_t hash_pos(uint32_t v, uint32_t b5) {
    return (b5 * 0x9E3779u + v * 2654435761u) >> (32 - kHashLog);
}

// The walk's next landing after a match ending at step-relative position np: the first matched
// lane of the step mask mq probing at or after np, or 64 when there is none in this step
template <uint32_t kPSt>
__device__ __forceinline__ uint32_t next_landing(uint64_t mq, uint32_t np) {
    const uint32_t kk = (np + kPSt - 1u) / kPSt;
    const uint64_t rest = kk < 64u ? mq >> kk : 0ull;
    const uint32_t lo = (uint32_t)rest, hi = (uint32_t)(rest >> 32);
    const uint32_t tz = lo ? (uint32_t)__builtin_ctz(lo) : 32u + (uint32_t)__builtin_ctz(hi | 0x80000000u);
    return rest ? kk + tz : 64u;
}

// Stage block bytes [lo, hi) into lds (lds[x - lo]); any alignment. Every lane issues all of
// its loads (8 x 16 B per pass) before the first LDS store, so staging costs one HBM round trip
// per 8 KiB instead of one per dword.
__device__ void stage_in(const uint8_t* blk, uint32_t lo, uint32_t hi, uint8_t* lds, uint32_t lane, uint32_t nthr) {
    const uint32_t n = hi - lo;
    const uint8_t* g = blk + lo;
    const uint32_t nv = n >> 4;  // whole 16-byte vectors
    if (nv && (((uintptr_t)g) & 15) == 0) {
        const uint4* sv = (const uint4*)g;
        for (uint32_t base = 0; base < nv; base += nthr * 8) {
            // loads are unconditional (clamped index) so the group stays in registers
            uint4 v0, v1, v2, v3, v4, v5, v6, v7;
#define S3HC_LD(q, vq) { const uint32_t j = base + lane + nthr * q; vq = sv[j < nv ? j : nv - 1]; }
            S3HC_LD(0, v0) S3HC_LD(1, v1) S3HC_LD(2, v2) S3HC_LD(3, v3)
            S3HC_LD(4, v4) S3HC_LD(5, v5) S3HC_LD(6, v6) S3HC_LD(7, v7)
#undef S3HC_LD
#define S3HC_ST(q, vq) { const uint32_t j = base + lane + nthr * q; if (j < nv) *(uint4*)(lds + 16 * j) = vq; }
            S3HC_ST(0, v0) S3HC_ST(1, v1) S3HC_ST(2, v2) S3HC_ST(3, v3)
            S3HC_ST(4, v4) S3HC_ST(5, v5) S3HC_ST(6, v6) S3HC_ST(7, v7)
#undef S3HC_ST
        }
    } else if (nv) {
        const uintptr_t a = (uintptr_t)g & ~(uintptr_t)3;
        const uint32_t sh = (uint32_t)((uintptr_t)g & 3);
        const uint32_t* sw = (const uint32_t*)a;
        for (uint32_t base = 0; base < nv; base += nthr * 2) {
            const uint32_t ja = base + lane, jb = base + lane + nthr;
            const uint32_t ka = ja < nv ? ja : nv - 1, kb = jb < nv ? jb : nv - 1;
            const uint32_t a0 = sw[4 * ka], a1 = sw[4 * ka + 1], a2 = sw[4 * ka + 2], a3 = sw[4 * ka + 3];
            const uint32_t a4 = sh ? sw[4 * ka + 4] : 0u;  // holds valid bytes only when sh != 0
            const uint32_t b0 = sw[4 * kb], b1 = sw[4 * kb + 1], b2 = sw[4 * kb + 2], b3 = sw[4 * kb + 3];
            const uint32_t b4 = sh ? sw[4 * kb + 4] : 0u;
            if (ja < nv)
                *(uint4*)(lds + 16 * ja) = make_uint4(__builtin_amdgcn_alignbyte(a1, a0, sh), __builtin_amdgcn_alignbyte(a2, a1, sh),
                                                      __builtin_amdgcn_alignbyte(a3, a2, sh), __builtin_amdgcn_alignbyte(a4, a3, sh));
            if (jb < nv)
                *(uint4*)(lds + 16 * jb) = make_uint4(__builtin_amdgcn_alignbyte(b1, b0, sh), __builtin_amdgcn_alignbyte(b2, b1, sh),
                                                      __builtin_amdgcn_alignbyte(b3, b2, sh), __builtin_amdgcn_alignbyte(b4, b3, sh));
        }
    }
    for (uint32_t t = 16 * nv + lane; t < n; t += nthr) lds[t] = g[t];
}

// Match finding for one 4 KiB segment per wave (the segment's 4 KiB prefix window is staged
// too and pre-inserted into the hash table). Per 512-position sub-block:
//   A  table pass: every position hashes its 4 bytes, reads the per-wave LDS table (u16
//      window positions; the most recent earlier position with that hash) and inserts
//      itself; the eight 64-position steps go back to back (reads only wait at use).
//      Distance 1..4 repeats are detected from the position's own bytes.
//   B  measure pass: both candidates (table, short distance) are verified and measured in
//      one LDS round trip per step — forward up to kFwd bytes, backward up to 4 — and the
//      longer kept; a ballot gives the step's match mask, the probe word stays in a VGPR.
//   C  greedy walk, per 64-position chunk, from registers: next match = lowest mask bit at
//      or after the greedy position (s_ff1), its word by v_readlane, long matches extended
//      wave-wide; the chunk's hops then become sequence records lane-parallel.
// Matches end inside the segment, so segments are independent; k_enc_sizes stitches them.
#ifdef S3HC_ENC_WPE  // diagnostic builds: cap VGPRs for S3HC_ENC_WPE waves per SIMD
#define S3HC_ENC_WPE_ATTR __attribute__((amdgpu_num_vgpr(512 / S3HC_ENC_WPE / 8 * 8)))
#else
#define S3HC_ENC_WPE_ATTR
#endif
template <uint32_t kPS, uint32_t kIns>
__global__ __launch_bounds__(enc::kGThreads, S3HC_ENC_MINWAVES) S3HC_ENC_WPE_ATTR void k_enc_parse(const uint8_t* __restrict__ src,
                                                              const EncBlock* __restrict__ blocks,
                                                              const uint2* __restrict__ groups, uint32_t ngroups,
                                                              uint32_t nxx, const uint64_t* __restrict__ fsrc_off,
                                                              const uint32_t* __restrict__ fsrc_len, uint32_t nframes,
                                                              uint32_t* __restrict__ fhash, uint2* __restrict__ recs,
                                                              SegSummary* __restrict__ summ) {
    using namespace enc;
    static_assert(kPS == 1 || kPS == 2, "probe stride 1 or 2");
    constexpr uint32_t kStepPos = 64 * kPS;                     // positions of one step
    constexpr uint32_t kPSteps = kSteps / kPS;                  // steps of a sub-block (64 x kSteps positions)
    __shared__ __attribute__((aligned(16))) uint8_t inb_raw[kGIn];
    __shared__ __attribute__((aligned(16))) uint16_t tbl_all[kGroupSegs][kTbl + 8];  // slot kTbl: sink
    __shared__ __attribute__((aligned(16))) uint2 stash_all[kGroupSegs][kStash + 8];  // hops of a sub-block (+ sink)
#ifdef S3HC_ENC_LDS_PAD  // diagnostic builds: extra LDS per workgroup to lower occupancy
    __shared__ uint8_t enc_pad[S3HC_ENC_LDS_PAD];
    if (ngroups == 0xFFFFFFFFu) ((volatile uint8_t*)enc_pad)[threadIdx.x] = 0;
#endif
    // The first nxx workgroups compute the frames' content xxh32 (they are dispatched first and
    // overlap the match finding; the emitter reads the hashes).
    if (blockIdx.x < nxx) {
#ifndef S3HC_ENC_NOXXH  // diagnostic builds (timing only, frame checksums wrong): no content hashing
        xxh32_ranges_dev<32, false>(src, fsrc_off, fsrc_len, nframes, fhash, blockIdx.x * kGThreads + threadIdx.x);
#endif
        return;
    }
    const uint32_t gi = blockIdx.x - nxx;
    if (gi >= ngroups) return;
    // A group = up to kGroupSegs consecutive segments of one block, one wave each, sharing one
    // staged copy of the group's input and the 4 KiB window before it.
    const uint2 G = groups[gi];
    const EncBlock B = blocks[G.x];
    const uint32_t U = B.len;
    const uint32_t ns = B.nseg - G.y < kGroupSegs ? B.nseg - G.y : kGroupSegs;
    const uint32_t g_lo = G.y * kSeg;
    const uint32_t g_hi = g_lo + ns * kSeg < U ? g_lo + ns * kSeg : U;
    const uint32_t stage_lo = g_lo > kPrewarm ? g_lo - kPrewarm : 0;
    const uint32_t stage_hi = g_hi + 64 < U ? g_hi + 64 : U;
    const uint8_t* bin = src + B.src_off;
    const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int lane = lane_id();
    uint16_t* tbl = tbl_all[wv];
    uint2* stash = stash_all[wv];
    for (uint32_t t = lane; t < (kTbl + 8) / 8; t += 64) ((uint4*)tbl)[t] = make_uint4(~0u, ~0u, ~0u, ~0u);
    stage_in(bin, stage_lo, stage_hi, inb_raw + kPad, threadIdx.x, kGThreads);
    __syncthreads();
    if (wv >= ns) return;  // no barrier below
#ifdef S3HC_PROF
    uint64_t epr[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    const uint64_t tk0 = PROF_NOW();
#endif
    const uint32_t k = G.y + wv;
    const uint32_t s = B.seg0 + k;
    const uint32_t seg_lo = k * kSeg;
    const uint32_t seg_hi = seg_lo + kSeg < U ? seg_lo + kSeg : U;
    const uint32_t pw_lo = seg_lo > kPrewarm ? seg_lo - kPrewarm : 0;
    uint8_t* inb = inb_raw + kPad + (pw_lo - stage_lo);  // inb[x - pw_lo] = block byte x
    const uint32_t* dw = (const uint32_t*)inb;          // dw[-2 .. -1]: pad or earlier bytes
    const uint32_t ia_max = kGIn - kPad - (pw_lo - stage_lo) - 8;  // last safe lds32u index
    // Largest match end / start (LZ4: the last 5 bytes are literals and the last match starts
    // at least 12 bytes before the block end; segment matches end inside the segment).
    const uint32_t blk_end_lim = U >= 5 ? U - 5 : 0;
    const uint32_t end_lim = seg_hi < blk_end_lim ? seg_hi : blk_end_lim;
    int64_t smax = (int64_t)end_lim - 4;
    if ((int64_t)U - 12 < smax) smax = (int64_t)U - 12;
    // prewarm the table with the window before the segment
    // (four positions per lane from one aligned 8-byte read)
    {
        const uint32_t lim = seg_lo - pw_lo;  // window position i is inserted when i + 4 <= lim
        for (uint32_t d0 = lane; 4 * d0 < lim; d0 += 64) {
            const uint32_t w0 = dw[d0], w1 = dw[d0 + 1];
#pragma unroll
            for (uint32_t j = 0; j < 4; ++j) {
                const uint32_t i = 4 * d0 + j;
                tbl[i + 4 <= lim ? hash_pos(__builtin_amdgcn_alignbyte(w1, w0, j), __builtin_amdgcn_ubfe(w1, 8 * j, 8)) : kTbl] = (uint16_t)i;
            }
        }
    }
    wave_sync();
#ifdef S3HC_PROF
    epr[0] = PROF_NOW() - tk0;
#endif
    uint32_t x = seg_lo;         // greedy position (no match starts in [last_end, x))
    uint32_t last_end = seg_lo;  // end of the last recorded match (literal start)
    uint32_t nseq = 0, body = 0, ll0 = 0;
    uint2* myrec = recs + (size_t)s * kMaxSeqPerSeg;
    const uint32_t pend = smax < (int64_t)seg_lo ? seg_lo : (uint32_t)(smax + 1);  // probe [seg_lo, pend)
    for (uint32_t sb = seg_lo; sb < pend; sb += 64 * kSteps) {
        const uint32_t sb_end = sb + 64 * kSteps < pend ? sb + 64 * kSteps : pend;
        const uint64_t tc0 = PROF_NOW();
        PROF_ADD(epr, 6, 1);
        // ---- A: table pass
        uint32_t vv[kPSteps], vm[kPSteps], vm8[kPSteps], cc[kPSteps];
#pragma unroll
        for (uint32_t q = 0; q < kPSteps; ++q) {
            const uint32_t P = sb + kStepPos * q + kPS * lane;
            const uint32_t i = P - pw_lo;
            const uint32_t a = i >> 2, sh = i & 3;
            const uint32_t w0 = dw[a], w1 = dw[a + 1], wp = dw[(int)a - 1], wpp = dw[(int)a - 2];
            vv[q] = __builtin_amdgcn_alignbyte(w1, w0, sh);
            vm[q] = __builtin_amdgcn_alignbyte(w0, wp, sh);    // bytes [P-4, P)
            vm8[q] = __builtin_amdgcn_alignbyte(wp, wpp, sh);  // bytes [P-8, P-4)
            const uint32_t h = hash_pos(vv[q], __builtin_amdgcn_ubfe(w1, 8 * sh, 8));
            if (kPS == 1) {
                cc[q] = tbl[h];
                if constexpr (kIns != 0) {
                    if ((P < sb_end) & ((P & kIns) == 0)) tbl[h] = (uint16_t)i;  // exec-masked: no sink conflicts
                } else {
                    tbl[P < sb_end ? h : kTbl] = (uint16_t)i;
                }
            } else {
                // (i even: sh + 1 <= 3) the lane's second position is inserted after the first; the
                // two half-waves (64 positions each) read and insert one after the other, so a
                // probe sees every position before its own 64 (as with one position per lane)
                const uint32_t h1 = hash_pos(__builtin_amdgcn_alignbyte(w1, w0, sh + 1), __builtin_amdgcn_ubfe(w1, 8 * (sh + 1), 8));
                const uint32_t t0 = P < sb_end ? h : kTbl, t1 = P + 1 < sb_end ? h1 : kTbl;
#pragma unroll
                for (uint32_t half = 0; half < 2; ++half) {
                    if (((uint32_t)lane >> 5) == half) {
                        cc[q] = tbl[h];
                        tbl[t0] = (uint16_t)i;
                        tbl[t1] = (uint16_t)(i + 1);
                    }
                    wave_sync();
                }
            }
        }
        // ---- B: verify + measure both candidates (table: one LDS round trip; distance 1..4:
        // from the position's own bytes, no reads)
        uint32_t word[kPSteps], flen[kPSteps];
        uint64_t mm[kPSteps];
#pragma unroll
        for (uint32_t q = 0; q < kPSteps; ++q) {
            const uint32_t P = sb + kStepPos * q + kPS * lane;
            const bool valid = P < sb_end;
            const uint32_t i = P - pw_lo;
            const uint32_t v = vv[q], vm4 = vm[q];
            const bool e1 = __builtin_amdgcn_alignbyte(v, vm4, 3) == v, e2 = __builtin_amdgcn_alignbyte(v, vm4, 2) == v;
            const bool e3 = __builtin_amdgcn_alignbyte(v, vm4, 1) == v, e4 = vm4 == v;
#ifndef S3HC_SHORT_CAND
#define S3HC_SHORT_CAND 1
#endif
            const uint32_t c16 = cc[q];
#if S3HC_SHORT_CAND == 2
            // One candidate per position: where the bytes [P-4-d, P+4) repeat with a period d of
            // 1..4 (runs, padding, repeated separators) the candidate is P - d, otherwise the
            // table's. Decided from bytes already in registers, so the candidate read is not
            // delayed and only one candidate is measured.
            const uint32_t dfs = (e1 & (i >= 5u)) ? 1u : ((e2 & (i >= 6u)) ? 2u : ((e3 & (i >= 7u)) ? 3u : ((e4 & (i >= 8u)) ? 4u : 0u)));
            const bool per = (dfs != 0u) & (__builtin_amdgcn_alignbyte(vm4, vm8[q], (4u - dfs) & 3u) == vm4);
            const bool tin = per | ((c16 != kEmpty) & (c16 < i));
            const uint32_t ct = per ? i - dfs : (tin ? c16 : i);
#else
            const bool tin = (c16 != kEmpty) & (c16 < i);
            const uint32_t ct = tin ? c16 : i;
#endif
            const uint32_t a = i >> 2, sh = i & 3, ta = ct >> 2, ts = ct & 3;
            uint32_t O[kNQ + 1], T[kNQ + 3];
#pragma unroll
            for (int j = 0; j < kNQ + 1; ++j) O[j] = dw[a + 1 + j];
#pragma unroll
            for (int j = 0; j < kNQ + 3; ++j) T[j] = dw[(int)ta - 1 + j];
            uint32_t Q[kNQ + 1];  // Q[k] = bytes [P+4k, P+4k+4)
            Q[0] = v;
#pragma unroll
            for (int j = 0; j < kNQ; ++j) Q[j + 1] = __builtin_amdgcn_alignbyte(O[j + 1], O[j], sh);
            const uint32_t maxf = end_lim - P;  // >= 4 for P <= smax
            uint32_t dtt[kNQ];
#pragma unroll
            for (int j = 0; j < kNQ; ++j) dtt[j] = Q[j + 1] ^ __builtin_amdgcn_alignbyte(T[j + 3], T[j + 2], ts);
            uint32_t lt = umin32(umin32(fwd_len(dtt), kFwd), maxf);
            const uint32_t bt = vm4 ^ __builtin_amdgcn_alignbyte(T[1], T[0], ts);
            const uint32_t nbt = umin32(umin32(ffbh_hw(bt) >> 3, 4u), ct);  // ct < i
            const bool gt = valid & tin & (__builtin_amdgcn_alignbyte(T[2], T[1], ts) == v);
            uint32_t len = lt, nb = nbt, dist = i - ct;
            bool gf = false;
#ifndef S3HC_SHORT_MIN
#define S3HC_SHORT_MIN 24  // > kFwd: measured whenever a period 1..4 is seen (16: 1 % slower, same ratio)
#endif
            // the distance-1..4 candidate is measured only where the table candidate is absent
            // or shorter than S3HC_SHORT_MIN bytes (a long table match is kept as is)
#if S3HC_SHORT_GATE
            // the distance-1..4 candidate only where the table has no verified candidate (a run's
            // first positions: inside a run the table candidate lies in the run and measures the
            // same); the step's ballot then fires far less often
            bool want_short = valid & (e1 | e2 | e3 | e4) & !gt;
#else
            bool want_short = valid & (e1 | e2 | e3 | e4) & !(gt & (lt >= S3HC_SHORT_MIN));
#endif
#if S3HC_ABL == 2  // diagnostic ablation: no distance-1..4 candidate
            want_short = false;
#endif
            if (S3HC_SHORT_CAND == 1 && __ballot(want_short)) {
                const uint32_t df = (e1 & (i >= 1)) ? 1u : ((e2 & (i >= 2)) ? 2u : ((e3 & (i >= 3)) ? 3u : ((e4 & (i >= 4)) ? 4u : 0u)));
                gf = want_short & (df != 0);
                const uint32_t fs = (4u - df) & 3u;
                uint32_t dff[kNQ];
#pragma unroll
                for (int j = 0; j < kNQ; ++j) dff[j] = Q[j + 1] ^ __builtin_amdgcn_alignbyte(Q[j + 1], Q[j], fs);
                const uint32_t lf = umin32(umin32(fwd_len(dff), kFwd), maxf);
                const uint32_t bf = vm4 ^ __builtin_amdgcn_alignbyte(vm4, vm8[q], fs);
                const uint32_t nbf = umin32(umin32(ffbh_hw(bf) >> 3, 4u), i - df);
                const bool ut = gt & (!gf | (lt >= lf));
                len = ut ? lt : lf;
                nb = ut ? nbt : nbf;
                dist = ut ? i - ct : df;
            }
            word[q] = dist | ((len - 4) << 16) | (nb << 24);
            flen[q] = len;
#if S3HC_LAZY
            // Lazy selection, off the walk's chain: a match is left out of the step's mask when the
            // next position's match is longer (and it is not a wave-extended one); the walk then
            // lands on the next one, so a run of growing matches lands on its longest. One literal
            // buys >= 1 more matched byte: config 2's C/U 0.387 -> 0.379, fewer sequences to decode.
            const uint32_t fv = (gt | gf) ? len : 0u;
            const uint32_t fnext = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)fv, 0x130, 0xF, 0xF, false);  // wave_shl:1
            mm[q] = __ballot((gt | gf) & !((fnext > fv) & (fv < kFwd)));
#else
            mm[q] = __ballot(gt | gf);
#endif
#if S3HC_SALU_PAD  // diagnostic: extra scalar instructions per step (scalar-unit sensitivity)
            {
                uint32_t d0 = q;
#pragma unroll
                for (int k = 0; k < S3HC_SALU_PAD; ++k) asm volatile("s_add_u32 %0, %0, 1" : "+s"(d0));
                asm volatile("" ::"s"(d0));
            }
#endif
#if S3HC_VALU_PAD  // diagnostic: extra vector instructions per step (VALU sensitivity)
            {
                uint32_t d1 = lane;
#pragma unroll
                for (int k = 0; k < S3HC_VALU_PAD; ++k) asm volatile("v_add_u32 %0, %0, 1" : "+v"(d1));
                asm volatile("" ::"v"(d1));
            }
#endif
            if (q & 1) wave_sync();  // bounds the loads hoisted ahead (VGPR pressure)
        }
        const uint64_t tc1 = PROF_NOW();
        PROF_ADD(epr, 1, tc1 - tc0);
        // ---- C: greedy walk over the chunks (scalar); each chunk's hops are stashed in LDS in
        // order, then the sub-block's sequence records are formed 64 hops at a time
        const uint32_t ns_sb = nseq, le_sb = last_end;
        WALK_PRIO_ON();
#pragma unroll
        for (uint32_t q = 0; q < kPSteps; ++q) {
            const uint32_t base = sb + kStepPos * q;
            if (x >= base + kStepPos || !mm[q]) continue;
            uint64_t hm = 0;
            const uint64_t mq = mm[q];
            // per lane: the walk's move after taking this lane's match: the next landing's lane
            // (< 64) when one lies in this step; else 0x100 | the step-relative position after the
            // match (it leaves the step, or no match follows it here); 0x80 for a match that
            // reached kFwd (extended wave-wide first). A hop is one v_readlane, lane to lane.
            const uint32_t np = kPS * (uint32_t)lane + flen[q];
            const uint32_t nl = next_landing<kPS>(mq, np);
            const uint32_t nxl = flen[q] == kFwd ? 0x80u : (nl < 64u ? nl : 0x100u | np);
            uint32_t r = x > base ? x - base : 0u;  // < kStepPos
            // the first probed position at or after r (a probe after r reaches back to it)
            uint32_t j0 = (r + kPS - 1u) / kPS;
            uint64_t av = j0 < 64u ? mq & (~0ull << j0) : 0ull;
#if S3HC_ABL == 1  // diagnostic ablation: no serial walk (frames not valid)
            hm = mq & 0x1111111111111111ull;
            r = kStepPos;
            av = 0;
#endif
            while (av) {
                uint32_t j = (uint32_t)__builtin_ctzll(av);
                uint32_t v;
                for (;;) {
                    hm |= 1ull << j;
                    v = rdl(nxl, j);
                    if (v >= 64u) break;
                    j = v;
                }
                if (v & 0x100u) {  // no further landing in this step
                    r = v & 0xFFu;
                    break;
                }
                {  // long match: wave-wide forward extension
                    const uint64_t tx0 = PROF_NOW();
                    PROF_ADD(epr, 8, 1);
                    const uint32_t wj = rdl(word[q], j);
                    const uint32_t P = base + kPS * j;
                    const uint32_t maxf = end_lim - P;
                    const uint32_t c = P - (wj & 0xFFFFu);
                    uint32_t lenf = kFwd;
                    while (lenf < maxf) {
                        const uint32_t rel = lenf + 4u * lane;
                        uint32_t e2;
                        if (rel >= maxf) {
                            e2 = 0;
                        } else {
                            uint32_t ia = P + rel - pw_lo;
                            if (ia > ia_max) ia = ia_max;
                            const uint32_t xa = lds32u(inb, ia), ya = lds32u(inb, c + rel - pw_lo);
                            e2 = xa == ya ? 4u : (uint32_t)__builtin_ctz(xa ^ ya) >> 3;
                            if (e2 > maxf - rel) e2 = maxf - rel;
                        }
                        const uint64_t m2 = __ballot(e2 != 4u);
                        if (m2 == 0) { lenf += 256; continue; }
                        const uint32_t g = (uint32_t)__builtin_ctzll(m2);
                        lenf += 4u * g + rdl(e2, g);
                        break;
                    }
                    flen[q] = (uint32_t)lane == j ? lenf : flen[q];
                    r = kPS * j + lenf;
                    PROF_ADD(epr, 2, PROF_NOW() - tx0);
                }
                j0 = (r + kPS - 1u) / kPS;
                av = j0 < 64u ? mq & (~0ull << j0) : 0ull;
            }
            x = base + r;
            if (hm) {
                const uint32_t rank =
                    __builtin_amdgcn_mbcnt_hi((uint32_t)(hm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)hm, 0));
                const uint32_t hidx = (hm >> lane) & 1ull ? nseq - ns_sb + rank : kStash + ((uint32_t)lane & 7u);
                stash[hidx] = make_uint2((base + kPS * lane - seg_lo) | (flen[q] << 16), word[q]);
                last_end = base + r;
                nseq += (uint32_t)__builtin_popcountll(hm);
            }
        }
        WALK_PRIO_OFF();
        const uint64_t tf0 = PROF_NOW();
        wave_sync();
        {
#if S3HC_ABL == 4  // diagnostic ablation: stash read once, no record formation
            const uint32_t H = 0;
            body += stash[lane].x + stash[lane].y;
#else
            const uint32_t H = nseq - ns_sb;
#endif
            uint32_t carry_end = le_sb;
            for (uint32_t g = 0; g < H; g += 64) {
                const uint32_t idx = g + lane;
                const bool act = idx < H;
                const uint2 e = stash[act ? idx : 0u];
                const uint32_t P = seg_lo + (e.x & 0xFFFFu), lenf = e.x >> 16, wd = e.y;
                const uint32_t endj = P + lenf;
                const uint32_t pe = dpp0<0x138, 0xF>(endj);  // wave_shr:1: previous hop's end
                const uint32_t prev = lane == 0 ? carry_end : pe;
                uint32_t nb = (wd >> 24) & 7u;
                nb = nb > P - prev ? P - prev : nb;
                const uint32_t ll = P - nb - prev;
                const uint32_t len = nb + lenf;
                const uint32_t gj = ns_sb + idx;
                const uint32_t tok = gj == 0 ? 0u : 1u + ext_bytes(ll);
                const uint32_t sz = act ? tok + ll + 2u + ext_bytes(len - 4) : 0u;
                body += rdl(wave_incl_sum(sz), 63);
                if (ns_sb == 0 && g == 0) ll0 = rdl(ll, 0);  // first sequence of the segment
                if (act) myrec[gj] = make_uint2(ll | (len << 16), wd & 0xFFFFu);
                const uint32_t last = H - g < 64 ? H - g - 1 : 63u;
                carry_end = rdl(endj, last);
            }
        }
        wave_sync();
        PROF_ADD(epr, 4, PROF_NOW() - tf0);
        PROF_ADD(epr, 3, PROF_NOW() - tc1);
    }
#ifdef S3HC_PROF
    epr[5] = PROF_NOW() - tk0;
    epr[7] = nseq;
    if (lane == 0)
        for (int q = 0; q < 9; ++q) atomicAdd(&g_prof[16 + q], (unsigned long long)epr[q]);
#endif
    if (lane == 0) {
        SegSummary S;
#if S3HC_ABL == 1 || S3HC_ABL == 4  // ablations: the segment is written as literals (safe sizes)
        nseq = 0;
#endif
        S.nseq = nseq;
        S.ll0 = ll0;
        S.body = body;
        S.trail = seg_hi - last_end;
        summ[s] = S;
    }
}

// One thread per block: stitch segment carries, size the payload, decide stored/compressed.
__global__ void k_enc_sizes(const EncBlock* __restrict__ blocks, uint32_t nblocks,
                            const SegSummary* __restrict__ summ, SegPlace* __restrict__ place,
                            uint32_t* __restrict__ blk_payload, uint32_t* __restrict__ blk_size,
                            uint32_t* __restrict__ blk_carry) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nblocks) return;
    const EncBlock B = blocks[b];
    const uint32_t hdr = (B.flags & EB_FIRST) ? 7u : 0u;
    const uint32_t trl = (B.flags & EB_LAST) ? 8u : 0u;
    if (B.flags & EB_EMPTY) {
        blk_payload[b] = 0;
        blk_size[b] = hdr + trl;
        blk_carry[b] = 0;
        return;
    }
    uint32_t payload = B.len;
    bool stored = true;
    uint32_t carry = 0;
    if (!(B.flags & EB_STORE)) {
        uint32_t off = 0;
        for (uint32_t k = 0; k < B.nseg; ++k) {
            const SegSummary S = summ[B.seg0 + k];
            const uint32_t lo = k * kSeg;
            const uint32_t hi = lo + kSeg < B.len ? lo + kSeg : B.len;
            SegPlace P;
            P.out_off = off;
            P.carry = carry;
            place[B.seg0 + k] = P;
            if (S.nseq == 0) {
                carry += hi - lo;
                continue;
            }
            const uint32_t lle = carry + S.ll0;
            off += 1 + ext_bytes(lle) + carry + S.body;
            carry = S.trail;
        }
        off += 1 + ext_bytes(carry) + carry;
        if (off < B.len) {  // lz4_flex write_block: Compressed iff comp_len < src.len()
            stored = false;
            payload = off;
        }
    }
    blk_payload[b] = payload | (stored ? kStoredBit : 0u);
    blk_size[b] = hdr + 4 + payload + trl;
    blk_carry[b] = carry;
}

// One wave per segment: write this segment's share of the framed output.
__global__ __launch_bounds__(256) void k_enc_emit(const uint8_t* __restrict__ src,
                                                  const EncBlock* __restrict__ blocks,
                                                  const uint32_t* __restrict__ seg_block, uint32_t nseg,
                                                  const uint2* __restrict__ recs,
                                                  const SegSummary* __restrict__ summ,
                                                  const SegPlace* __restrict__ place,
                                                  const uint32_t* __restrict__ blk_payload,
                                                  const uint32_t* __restrict__ blk_carry,
                                                  const uint64_t* __restrict__ blk_off,
                                                  const uint32_t* __restrict__ frame_hash, uint8_t* dst) {
    // Encoded body bound of one segment: a record consuming ll + ml input bytes (ml >= 4) emits
    // [j > 0](1 + ext(ll)) + ll + 2 + ext(ml - 4) bytes, i.e. at most ext(ll) - 1 more than it
    // consumes (2 + ext(ml - 4) - ml <= -2), and ext(ll) - 1 <= ll / 255; records consume at
    // most kSeg bytes, so the body is <= kSeg + kSeg / 255 (+ slack).
    constexpr uint32_t kOut = kSeg + 256;
    constexpr uint32_t kIb = kSeg + 64;
    constexpr uint32_t kWaveLds = kOut + kIb;
    __shared__ __attribute__((aligned(16))) uint8_t smem[2 * kWaveLds];
    const int lane = lane_id();
    const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const uint32_t s = blockIdx.x * 2 + wv;
    if (s >= nseg) return;
    uint8_t* ob = smem + wv * kWaveLds;
    uint8_t* ib = ob + kOut;
    const uint32_t b = seg_block[s];
    const EncBlock B = blocks[b];
    const uint32_t k = s - B.seg0;
    uint8_t* fo = dst + blk_off[b];
    const uint32_t hdr = (B.flags & EB_FIRST) ? 7u : 0u;
    const uint32_t pw = blk_payload[b];
    const bool stored = (pw & kStoredBit) != 0;
    const uint32_t payload = pw & ~kStoredBit;
    const uint32_t fh = frame_hash[B.frame];
    if (k == 0 && lane == 0) {
        if (B.flags & EB_FIRST) {
            fo[0] = 0x04; fo[1] = 0x22; fo[2] = 0x4D; fo[3] = 0x18;
            fo[4] = kFlgIndependentChecksum; fo[5] = B.bd; fo[6] = B.hc;
        }
        if (!(B.flags & EB_EMPTY)) {
            const uint32_t word = stored ? (B.len | kStoredBit) : payload;
            fo[hdr + 0] = (uint8_t)word; fo[hdr + 1] = (uint8_t)(word >> 8);
            fo[hdr + 2] = (uint8_t)(word >> 16); fo[hdr + 3] = (uint8_t)(word >> 24);
        }
    }
    const bool last_seg = k + 1 == B.nseg;
    if ((B.flags & EB_LAST) && last_seg && lane < 8) {
        const uint32_t tpos = (B.flags & EB_EMPTY) ? hdr : hdr + 4 + payload;
        const uint32_t v = lane < 4 ? 0u : fh;
        fo[tpos + lane] = (uint8_t)(v >> (8 * (lane & 3)));
    }
    if (B.flags & EB_EMPTY) return;
    uint8_t* pay = fo + hdr + 4;
    const uint32_t seg_lo = k * kSeg;
    const uint32_t seg_hi = seg_lo + kSeg < B.len ? seg_lo + kSeg : B.len;
    const uint8_t* bin = src + B.src_off;
    if (stored) {
        wave_copy_global(pay + seg_lo, bin + seg_lo, seg_hi - seg_lo, lane);
        return;
    }
    const SegSummary S = summ[s];
    const SegPlace P = place[s];
    uint32_t o = P.out_off;  // payload-relative write cursor
    if (S.nseq > 0) {
        const uint2* rr = recs + (size_t)s * kMaxSeqPerSeg;
        // the first four groups' records are loaded now, in flight with the input staging
        // below (each group used to wait for its own records: one HBM round trip per group)
        auto ldr = [&](uint32_t k) -> uint2 {
            const uint32_t jk = 64u * k + (uint32_t)lane;
            return rr[jk < S.nseq ? jk : 0u];
        };
        const uint2 pre0 = ldr(0), pre1 = ldr(1), pre2 = ldr(2), pre3 = ldr(3);
        const uint32_t ml0 = rdl(pre0.x, 0) >> 16;
        // first token: literal run = carry bytes (earlier segments) + ll0 (this segment)
        const uint32_t lle = P.carry + S.ll0;
        const uint32_t ne = ext_bytes(lle);
        if (lane == 0) {
            const uint32_t mn = ml0 - 4;
            pay[o] = (uint8_t)(((lle < 15 ? lle : 15) << 4) | (mn < 15 ? mn : 15));
        }
        for (uint32_t e = lane; e < ne; e += 64) pay[o + 1 + e] = e + 1 < ne ? 255 : (uint8_t)((lle - 15) % 255);
        o += 1 + ne;
        wave_copy_global(pay + o, bin + seg_lo - P.carry, P.carry, lane);
        o += P.carry;
        // body: records -> LDS, then one coalesced store
        stage_in(bin, seg_lo, seg_hi, ib, lane, 64);
        wave_sync();
        uint32_t ob_len = 0;   // bytes assembled in ob
        uint32_t in_pos = 0;   // segment-relative input cursor
        for (uint32_t g = 0; g < S.nseq; g += 64) {
            const uint32_t j = g + lane;
            const bool act = j < S.nseq;
            uint2 r = g == 0 ? pre0 : (g == 64 ? pre1 : (g == 128 ? pre2 : pre3));
            if (g >= 256u) r = act ? rr[j] : make_uint2(0, 0);
            if (!act) r = make_uint2(0, 0);
            const uint32_t ll = r.x & 0xFFFFu, ml = r.x >> 16, off = r.y;
            const uint32_t hsz = j == 0 ? 0u : 1 + ext_bytes(ll);
            const uint32_t sz = act ? hsz + ll + 2 + ext_bytes(ml - 4) : 0u;
            const uint32_t opos = ob_len + wave_excl_scan(sz, lane);
            const uint32_t ipos = in_pos + wave_excl_scan(act ? ll + ml : 0u, lane);
            const uint32_t tot = rdl(opos + sz, 63) - ob_len;                 // this group's bytes
            const uint32_t itot = rdl(ipos + (act ? ll + ml : 0u), 63) - in_pos;
            // literal runs of <= 48 bytes first, as 16-byte chunks of plain byte stores: last
            // chunk first, last byte first, so bytes past a lane's run (its offset and length
            // bytes, or later lanes' bytes) are always stored again after them (the record
            // bytes below; a later lane's chunk by a later store); longer runs are copied
            // wave-wide after the records
            const uint32_t lw = opos + hsz;  // my literals' position in ob
            const uint32_t nck = act && ll <= 48 ? (ll + 15u) >> 4 : 0u;
#pragma unroll
            for (int kc = 2; kc >= 0; --kc) {
                if (!__ballot(nck > (uint32_t)kc)) continue;
                if (nck > (uint32_t)kc) {
                    const uint32_t si = ipos + 16u * (uint32_t)kc, sa = si >> 2, sh = si & 3u;
                    const uint32_t* iw = (const uint32_t*)ib;
                    const uint32_t d0 = iw[sa], d1 = iw[sa + 1], d2 = iw[sa + 2], d3 = iw[sa + 3], d4 = iw[sa + 4];
                    const uint32_t x[4] = {__builtin_amdgcn_alignbyte(d1, d0, sh), __builtin_amdgcn_alignbyte(d2, d1, sh),
                                           __builtin_amdgcn_alignbyte(d3, d2, sh), __builtin_amdgcn_alignbyte(d4, d3, sh)};
                    uint8_t* dp = ob + lw + 16u * (uint32_t)kc;
#pragma unroll
                    for (int k = 15; k >= 0; --k) {
                        dp[k] = (uint8_t)(x[k >> 2] >> (8 * (k & 3)));
                        __builtin_amdgcn_sched_barrier(0);  // (the stores' order is the contract)
                    }
                }
            }
            wave_sync();
            if (act) {
                uint32_t w = opos;
                if (j != 0) {
                    const uint32_t mn = ml - 4;
                    ob[w++] = (uint8_t)(((ll < 15 ? ll : 15) << 4) | (mn < 15 ? mn : 15));
                    if (ll >= 15) {
                        uint32_t x = ll - 15;
                        while (x >= 255) { ob[w++] = 255; x -= 255; }
                        ob[w++] = (uint8_t)x;
                    }
                }
                w += ll;
                ob[w++] = (uint8_t)off;
                ob[w++] = (uint8_t)(off >> 8);
                if (ml - 4 >= 15) {
                    uint32_t x = ml - 4 - 15;
                    while (x >= 255) { ob[w++] = 255; x -= 255; }
                    ob[w++] = (uint8_t)x;
                }
            }
            // long literal runs: wave-cooperative copy, one record at a time
            uint64_t longm = __ballot(act && ll > 48);
            while (longm) {
                const uint32_t l = (uint32_t)__builtin_ctzll(longm);
                longm &= longm - 1;
                const uint32_t lll = rdl(ll, l), lo = rdl(opos, l) + rdl(hsz, l), li = rdl(ipos, l);
                for (uint32_t t = lane; t < lll; t += 64) ob[lo + t] = ib[li + t];
            }
            wave_sync();
            ob_len += tot;
            in_pos += itot;
        }
        wave_store_from_lds(pay + o, ob, ob_len, lane);
        o += ob_len;
    }
    if (last_seg) {
        const uint32_t L = blk_carry[b];
        const uint32_t ne = ext_bytes(L);
        if (lane == 0) pay[o] = (uint8_t)((L < 15 ? L : 15) << 4);
        for (uint32_t e = lane; e < ne; e += 64) pay[o + 1 + e] = e + 1 < ne ? 255 : (uint8_t)((L - 15) % 255);
        o += 1 + ne;
        wave_copy_global(pay + o, bin + B.len - L, L, lane);
    }
}

// Per frame: offset and framed length from the block table.
__global__ void k_enc_frames(const uint32_t* __restrict__ frame_blk0, const uint32_t* __restrict__ frame_nblk,
                             uint32_t nframes, const uint64_t* __restrict__ blk_off,
                             const uint32_t* __restrict__ blk_size, uint64_t* __restrict__ frame_off,
                             uint32_t* __restrict__ frame_len) {
    const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= nframes) return;
    const uint32_t b0 = frame_blk0[f], nb = frame_nblk[f];
    uint64_t len = 0;
    for (uint32_t i = 0; i < nb; ++i) len += blk_size[b0 + i];
    frame_off[f] = blk_off[b0];
    frame_len[f] = (uint32_t)len;
}

// Exclusive scan of u32 sizes into u64 offsets: single workgroup, chunked (n up to millions).
__device__ __forceinline__ void scan_u32_u64(const uint32_t* __restrict__ in, uint32_t n, uint64_t* __restrict__ out,
                                             uint64_t* __restrict__ total) {
    __shared__ uint64_t wsum[16];
    __shared__ uint64_t carry_s;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    if (t == 0) carry_s = 0;
    __syncthreads();
    for (uint32_t base = 0; base < n; base += 1024 * 4) {
        uint64_t v[4];
        uint64_t loc = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            uint32_t i = base + 4 * t + k;
            v[k] = i < n ? in[i] : 0;
            loc += v[k];
        }
        const uint64_t x = wave_incl_sum64(loc);
        if (lane == 63) wsum[wv] = x;
        __syncthreads();
        uint64_t wpre = 0;
        for (int k = 0; k < wv; ++k) wpre += wsum[k];
        uint64_t run = carry_s + wpre + x - loc;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            uint32_t i = base + 4 * t + k;
            if (i < n) out[i] = run;
            run += v[k];
        }
        __syncthreads();
        if (t == 1023) carry_s = run;
        __syncthreads();
    }
    if (t == 0) *total = carry_s;
}
__global__ __launch_bounds__(1024) void k_scan_u32_u64(const uint32_t* __restrict__ in, uint32_t n,
                                                       uint64_t* __restrict__ out, uint64_t* __restrict__ total) {
    scan_u32_u64(in, n, out, total);
}
// two independent scans of n entries in one launch (one workgroup each)
__global__ __launch_bounds__(1024) void k_scan2_u32_u64(const uint32_t* __restrict__ in0, const uint32_t* __restrict__ in1,
                                                        uint32_t n, uint64_t* __restrict__ out0,
                                                        uint64_t* __restrict__ out1, uint64_t* __restrict__ total) {
    if (blockIdx.x == 0) scan_u32_u64(in0, n, out0, total);
    else scan_u32_u64(in1, n, out1, total + 1);
}

// ============================================ device-side frame walk (decode)
// One thread per frame: validate the header (FrameInfo::read), walk block words, count blocks.
// Header/BD/HC rules follow lz4_flex frame/header.rs as restated in oracle/lz4_oracle.c.
__device__ __forceinline__ uint32_t rd32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
__device__ uint32_t xxh32_small(const uint8_t* p, uint32_t n) {  // n < 16 (frame header bytes)
    uint32_t h = XP5 + n, t = 0;
    while (t + 4 <= n) { h += rd32(p + t) * XP3; h = rotl32(h, 17) * XP4; t += 4; }
    while (t < n) { h += (uint32_t)p[t] * XP5; h = rotl32(h, 11) * XP1; t++; }
    h ^= h >> 15; h *= XP2; h ^= h >> 13; h *= XP3; h ^= h >> 16;
    return h;
}

struct FrameWalk {
    int status;
    uint32_t nblk;
    uint32_t bmax;
    uint32_t flg;
    uint32_t hdr;
    uint32_t end;        // bytes consumed by the frame (through its checksum)
    uint32_t want;       // expected content checksum
    uint32_t content_lo; // content size (low 32 bits) if FLG content-size bit
};

__device__ FrameWalk walk_frame(const uint8_t* f, uint32_t avail, DecBlock* out_blocks, uint64_t src_base,
                                uint64_t dst_base, uint32_t dst_cap, uint32_t frame, uint64_t tok_base = 0) {
    FrameWalk r = {S3HC_OK, 0, 0, 0, 0, 0, 0, 0};
    if (avail < 4) { r.status = S3HC_CORRUPT; return r; }
    const uint32_t magic = rd32(f);
    if (magic == 0x184C2102u || (magic & 0xFFFFFFF0u) == 0x184D2A50u) { r.status = S3HC_UNSUPPORTED; return r; }
    if (magic != kMagic || avail < 7) { r.status = S3HC_CORRUPT; return r; }
    const uint32_t flg = f[4], bd = f[5];
    uint32_t need = 7 + ((flg & 0x08) ? 8 : 0) + ((flg & 0x01) ? 4 : 0);
    if (avail < need || (flg & 0xC0) != 0x40 || (flg & 0x02) || (bd & 0x8F)) { r.status = S3HC_CORRUPT; return r; }
    const uint32_t code = (bd >> 4) & 7;
    if (code < 4) { r.status = S3HC_CORRUPT; return r; }
    const uint32_t bmax = 1u << (16 + 2 * (code - 4));
    if (((xxh32_small(f + 4, need - 5) >> 8) & 0xFF) != f[need - 1]) { r.status = S3HC_CORRUPT; return r; }
    if (flg & 0x01) { r.status = S3HC_UNSUPPORTED; return r; }
    r.flg = flg;
    r.bmax = bmax;
    r.hdr = need;
    if (flg & 0x08) r.content_lo = rd32(f + 6);
    uint32_t ip = need;
    uint32_t k = 0;
    for (;;) {
        if (avail - ip < 4) { r.status = S3HC_CORRUPT; return r; }
        const uint32_t w = rd32(f + ip);
        ip += 4;
        if (w == 0) {
            if (flg & 0x04) {
                if (avail - ip < 4) { r.status = S3HC_CORRUPT; return r; }
                r.want = rd32(f + ip);
                ip += 4;
            }
            break;
        }
        const uint32_t len = w & 0x7FFFFFFFu;
        if (len > bmax || avail - ip < len + ((flg & 0x10) ? 4u : 0u)) { r.status = S3HC_CORRUPT; return r; }
        if (out_blocks) {
            DecBlock D;
            D.src_off = src_base + ip;
            const uint64_t slot = (uint64_t)k * bmax;
            D.dst_off = dst_base + slot;
            D.csize = len;
            D.limit = (w & kStoredBit) ? len : bmax;
            const uint64_t room = slot < dst_cap ? dst_cap - slot : 0;
            D.cap = room < D.limit ? (uint32_t)room : D.limit;
            D.flags = ((w & kStoredBit) ? DB_STORED : 0u) | ((flg & 0x20) ? 0u : DB_LINKED);
            D.frame = frame;
            D.tok = (uint32_t)(tok_base + ip / 3u);  // (tok_frame_entries: disjoint per block)
            out_blocks[k] = D;
        }
        ip += len + ((flg & 0x10) ? 4u : 0u);
        k++;
    }
    r.nblk = k;
    r.end = ip;
    return r;
}

// Block slots per frame are bounded by dst_cap/64KiB + 2 (planner capacity); a frame with
// more blocks than that cannot land contiguously anyway and is reported UNSUPPORTED.
__global__ void k_dframe_count(const uint8_t* __restrict__ src, const uint64_t* __restrict__ frame_off,
                               const uint32_t* __restrict__ frame_len, const uint32_t* __restrict__ dst_cap,
                               uint32_t nframes, uint32_t* __restrict__ nblk, int32_t* __restrict__ fstatus) {
    const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= nframes) return;
    FrameWalk r = walk_frame(src + frame_off[f], frame_len[f], nullptr, 0, 0, 0, f);
    if (r.status == S3HC_OK && r.end != frame_len[f]) r.status = S3HC_CORRUPT;  // one frame per entry
    if (r.status == S3HC_OK && r.nblk > dst_cap[f] / 65536u + 2u) r.status = S3HC_UNSUPPORTED;
    nblk[f] = r.status == S3HC_OK ? r.nblk : 0u;
    fstatus[f] = r.status;
}

__global__ void k_dframe_fill(const uint8_t* __restrict__ src, const uint64_t* __restrict__ frame_off,
                              const uint32_t* __restrict__ frame_len, uint32_t nframes,
                              const uint64_t* __restrict__ dst_off, const uint32_t* __restrict__ dst_cap,
                              const uint64_t* __restrict__ blk_base, const int32_t* __restrict__ fstatus,
                              DecBlock* __restrict__ blocks, DecUnit* __restrict__ units,
                              uint32_t* __restrict__ fwant, const uint64_t* __restrict__ ftok) {
    const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= nframes) return;
    if (fstatus[f] != S3HC_OK) return;
    const uint32_t b0 = (uint32_t)blk_base[f];
    FrameWalk r = walk_frame(src + frame_off[f], frame_len[f], blocks + b0, frame_off[f], dst_off[f], dst_cap[f], f,
                             ftok[f]);
    fwant[f] = r.want;
    const bool linked = !(r.flg & 0x20);
    for (uint32_t k = 0; k < r.nblk; ++k) {
        DecUnit U;
        if (linked) { U.first = b0; U.n = k == 0 ? r.nblk : 0; }
        else { U.first = b0 + k; U.n = 1; }
        units[b0 + k] = U;
    }
}

// Per frame after block decode: status, decoded length, contiguity, checksum range.
__global__ void k_dframe_finish(const uint64_t* __restrict__ blk_base, uint32_t nframes,
                                const uint32_t* __restrict__ nblk, const DecBlock* __restrict__ blocks,
                                const uint32_t* __restrict__ blk_out, const int32_t* __restrict__ blk_status,
                                int32_t* __restrict__ fstatus, uint32_t* __restrict__ out_len) {
    const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= nframes) return;
    int st = fstatus[f];
    uint64_t tot = 0;
    if (st == S3HC_OK) {
        const uint32_t b0 = (uint32_t)blk_base[f], nb = nblk[f];
        for (uint32_t k = 0; k < nb; ++k) {
            const int bs = blk_status[b0 + k];
            if (bs != S3HC_OK) { st = bs; break; }
            const DecBlock D = blocks[b0 + k];
            // independent blocks decode into slots k*bmax; all but the last must be full
            if (!(D.flags & DB_LINKED) && k + 1 < nb && blk_out[b0 + k] != D.limit) { st = S3HC_UNSUPPORTED; break; }
            tot += blk_out[b0 + k];
        }
    }
    fstatus[f] = st;
    out_len[f] = st == S3HC_OK ? (uint32_t)tot : 0u;
}

__global__ void k_dframe_verify(const uint8_t* __restrict__ src, const uint64_t* __restrict__ frame_off,
                                uint32_t nframes, const uint32_t* __restrict__ fwant,
                                const uint32_t* __restrict__ got_hash, const uint32_t* __restrict__ out_len,
                                int32_t* __restrict__ fstatus) {
    const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= nframes) return;
    if (fstatus[f] != S3HC_OK) return;
    const uint8_t* fp = src + frame_off[f];
    const uint32_t flg = fp[4];
    if ((flg & 0x08) && (rd32(fp + 6) | ((uint64_t)rd32(fp + 10) << 32)) != out_len[f]) {
        fstatus[f] = S3HC_CORRUPT;
        return;
    }
    if ((flg & 0x04) && got_hash[f] != fwant[f]) fstatus[f] = S3HC_CHECKSUM;
}

constexpr uint32_t kCloseLanes = 4;  // lanes per frame (16 per frame with DPP-shared P2 products measured slower)
// k_dframe_finish + k_xxh32_ranges + k_dframe_verify in one launch (same rules, same results):
// lanes 4f..4f+3 own frame f; each sums the frame's block results (frames hold few blocks), the
// four hash the frame's output, lane 4f checks the EndMark. fstat_in: statuses set before the
// decode (nullptr: none). blk_hash (nullable): hashes the large-block path computed while
// decoding (1 << 32 | xxh32 per block); a frame of one such block skips its own pass.
// got_hash (nullable): each frame's content xxh32.
// (lane gid of the close: frame gid / 4; callable by any workgroup shape whose lanes come in
// aligned groups of four)
__device__ __forceinline__ void dframe_close_lane(uint32_t gid, const uint8_t* __restrict__ src, const uint64_t* __restrict__ frame_off,
                                                  const uint64_t* __restrict__ blk_base, const uint32_t* __restrict__ nblk,
                                                  const DecBlock* __restrict__ blocks, const uint32_t* __restrict__ blk_out,
                                                  const int32_t* __restrict__ blk_status,
                                                  const uint64_t* __restrict__ blk_hash, const uint8_t* __restrict__ out,
                                                  const uint64_t* __restrict__ out_off, const uint32_t* __restrict__ fwant,
                                                  uint32_t n, const int32_t* fstat_in, int32_t* fstatus,
                                                  uint32_t* __restrict__ out_len, uint32_t* __restrict__ got_hash,
                                                  uint32_t* __restrict__ pend) {
    const uint32_t f = gid / kCloseLanes, j = gid % kCloseLanes;
    const bool act = f < n;
    int st = S3HC_OK;
    uint64_t tot = 0;
    uint64_t pre = 0;  // 1 << 32 | hash when the large-block path hashed the frame's only block
    if (act) {
        st = fstat_in ? fstat_in[f] : S3HC_OK;
        if (st == S3HC_OK) {
            const uint32_t b0 = (uint32_t)blk_base[f], nb = nblk[f];
            if (blk_hash && nb == 1) pre = blk_hash[b0];
            for (uint32_t k = 0; k < nb; ++k) {
                const int bs = blk_status[b0 + k];
                if (bs != S3HC_OK) { st = bs; break; }
                const DecBlock D = blocks[b0 + k];
                if (!(D.flags & DB_LINKED) && k + 1 < nb && blk_out[b0 + k] != D.limit) { st = S3HC_UNSUPPORTED; break; }
                tot += blk_out[b0 + k];
            }
        }
    }
    const uint32_t L = st == S3HC_OK ? (uint32_t)tot : 0u;
    const bool have = (pre >> 32) != 0;
    // pend (nullable): the range reader's first close of a batch (stream_range_data order,
    // disk_cache.rs:3884-3898: lz4_flex checks the content checksum at the EndMark, after the
    // frame's bytes were returned). A frame whose hash no decode kernel computed is left
    // unverified here (pend[f] = 1, status without the checksum); a second, full close of the same
    // frames follows on the queue and gives the final statuses behind the delivered bytes.
    const bool defer = pend && act && st == S3HC_OK && !have && (src[frame_off[f] + 4] & 0x04);
    uint32_t h = xxh32_lanes<32, true>(out + (act ? out_off[f] : 0), have || defer ? 0u : L, act, j);
    if (!act || j != 0) return;
    if (have) h = (uint32_t)pre;
    out_len[f] = L;
    if (got_hash) got_hash[f] = h;
    if (st == S3HC_OK) {
        const uint8_t* fp = src + frame_off[f];
        const uint32_t flg = fp[4];
        if ((flg & 0x08) && (rd32(fp + 6) | ((uint64_t)rd32(fp + 10) << 32)) != L) st = S3HC_CORRUPT;
        else if ((flg & 0x04) && !defer && h != fwant[f]) st = S3HC_CHECKSUM;
    }
    if (pend) pend[f] = defer && st == S3HC_OK ? 1u : 0u;
    fstatus[f] = st;
}
__global__ __launch_bounds__(64) void k_dframe_close(const uint8_t* __restrict__ src, const uint64_t* __restrict__ frame_off,
                                                     const uint64_t* __restrict__ blk_base, const uint32_t* __restrict__ nblk,
                                                     const DecBlock* __restrict__ blocks, const uint32_t* __restrict__ blk_out,
                                                     const int32_t* __restrict__ blk_status,
                                                     const uint64_t* __restrict__ blk_hash, const uint8_t* __restrict__ out,
                                                     const uint64_t* __restrict__ out_off, const uint32_t* __restrict__ fwant,
                                                     uint32_t n, const int32_t* fstat_in, int32_t* fstatus,
                                                     uint32_t* __restrict__ out_len, uint32_t* __restrict__ got_hash,
                                                     uint32_t* __restrict__ pend) {
    dframe_close_lane(blockIdx.x * blockDim.x + threadIdx.x, src, frame_off, blk_base, nblk, blocks, blk_out, blk_status,
                      blk_hash, out, out_off, fwant, n, fstat_in, fstatus, out_len, got_hash, pend);
}

}  // namespace s3hc

// ================================================================ launchers
// Host-side wrappers so the runtime (s3hc_runtime.cpp) never needs the kernel symbols.
namespace s3hc {
static inline uint32_t cdiv(uint64_t a, uint64_t b) { return (uint32_t)((a + b - 1) / b); }

hipError_t launch_xxh32(const uint8_t* base, const uint64_t* off, const uint32_t* len, uint32_t n, uint32_t* out,
                        hipStream_t st) {
    if (!n) return hipSuccess;
    // 16 ranges per 64-lane workgroup: 4096 frames spread over all 256 CUs instead of 64
    hipLaunchKernelGGL(k_xxh32_ranges, dim3(cdiv((uint64_t)n * 4, 64)), dim3(64), 0, st, base, off, len, n, out);
    return hipGetLastError();
}
hipError_t launch_decode_units(const uint8_t* src, uint8_t* dst, const DecBlock* blk, const DecUnit* units,
                               uint32_t nunits, const uint64_t* ucount, uint32_t grid, uint32_t* blk_out,
                               int32_t* blk_status, const uint8_t* unit_lb, const uint8_t* unit_fast, hipStream_t st) {
    if (!nunits || !grid) return hipSuccess;
#if S3HC_DIAG_VARIANTS
    // S3HC_DEC_ONEWAVE=1 (diagnostic builds): one wave per unit doing both halves (k_decode_units)
    if (knob_on(KN_DEC_ONEWAVE)) {
        hipLaunchKernelGGL(k_decode_units, dim3(cdiv(grid, dec::kWaves)), dim3(64 * dec::kWaves), 0, st, src, dst,
                           blk, units, nunits, ucount, blk_out, blk_status, unit_lb, unit_fast);
        return hipGetLastError();
    }
#endif
    hipLaunchKernelGGL(k_decode_pe, dim3(grid), dim3(128), 0, st, src, dst, blk, units, nunits, ucount, blk_out,
                       blk_status, unit_lb, unit_fast);
    return hipGetLastError();
}
hipError_t launch_enc_parse(const uint8_t* src, const EncBlock* blocks, const uint2* groups, uint32_t ngroups,
                            const uint64_t* fsrc_off, const uint32_t* fsrc_len, uint32_t nframes, uint32_t* fhash,
                            uint2* recs, SegSummary* summ, int mode, hipStream_t st) {
    const uint32_t nxx = cdiv((uint64_t)nframes * 4, enc::kGThreads);
    if (!ngroups && !nxx) return hipSuccess;
    if (mode == 1)  // S3HC_ENC_SMALL
        hipLaunchKernelGGL((k_enc_parse<1, 1>), dim3(nxx + ngroups), dim3(enc::kGThreads), 0, st, src, blocks, groups,
                           ngroups, nxx, fsrc_off, fsrc_len, nframes, fhash, recs, summ);
    else
        hipLaunchKernelGGL((k_enc_parse<2, 0>), dim3(nxx + ngroups), dim3(enc::kGThreads), 0, st, src, blocks, groups,
                           ngroups, nxx, fsrc_off, fsrc_len, nframes, fhash, recs, summ);
    return hipGetLastError();
}
hipError_t launch_enc_sizes(const EncBlock* blocks, uint32_t nblocks, const SegSummary* summ, SegPlace* place,
                            uint32_t* blk_payload, uint32_t* blk_size, uint32_t* blk_carry, hipStream_t st) {
    if (!nblocks) return hipSuccess;
    hipLaunchKernelGGL(k_enc_sizes, dim3(cdiv(nblocks, 256)), dim3(256), 0, st, blocks, nblocks, summ, place,
                       blk_payload, blk_size, blk_carry);
    return hipGetLastError();
}
hipError_t launch_scan(const uint32_t* in, uint32_t n, uint64_t* out, uint64_t* total, hipStream_t st) {
    hipLaunchKernelGGL(k_scan_u32_u64, dim3(1), dim3(1024), 0, st, in, n, out, total);
    return hipGetLastError();
}
hipError_t launch_scan2(const uint32_t* in0, const uint32_t* in1, uint32_t n, uint64_t* out0, uint64_t* out1,
                        uint64_t* total, hipStream_t st) {
    hipLaunchKernelGGL(k_scan2_u32_u64, dim3(2), dim3(1024), 0, st, in0, in1, n, out0, out1, total);
    return hipGetLastError();
}
hipError_t launch_enc_emit(const uint8_t* src, const EncBlock* blocks, const uint32_t* seg_block, uint32_t nseg,
                           const uint2* recs, const SegSummary* summ, const SegPlace* place,
                           const uint32_t* blk_payload, const uint32_t* blk_carry, const uint64_t* blk_off,
                           const uint32_t* frame_hash, uint8_t* dst, hipStream_t st) {
    if (!nseg) return hipSuccess;
    hipLaunchKernelGGL(k_enc_emit, dim3(cdiv(nseg, 2)), dim3(128), 0, st, src, blocks, seg_block, nseg, recs, summ,
                       place, blk_payload, blk_carry, blk_off, frame_hash, dst);
    return hipGetLastError();
}
hipError_t launch_enc_groups(const uint32_t* g_blk0, const uint32_t* g_nblk, uint32_t ng, const uint64_t* blk_off,
                             const uint32_t* blk_size, uint64_t* g_off, uint32_t* g_len, hipStream_t st) {
    if (!ng) return hipSuccess;
    hipLaunchKernelGGL(k_enc_frames, dim3(cdiv(ng, 256)), dim3(256), 0, st, g_blk0, g_nblk, ng, blk_off, blk_size,
                       g_off, g_len);
    return hipGetLastError();
}
hipError_t launch_dframe_count(const uint8_t* src, const uint64_t* frame_off, const uint32_t* frame_len,
                               const uint32_t* dst_cap, uint32_t n, uint32_t* nblk, int32_t* fstatus,
                               hipStream_t st) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_dframe_count, dim3(cdiv(n, 256)), dim3(256), 0, st, src, frame_off, frame_len, dst_cap, n,
                       nblk, fstatus);
    return hipGetLastError();
}
hipError_t launch_dframe_fill(const uint8_t* src, const uint64_t* frame_off, const uint32_t* frame_len, uint32_t n,
                              const uint64_t* dst_off, const uint32_t* dst_cap, const uint64_t* blk_base,
                              const int32_t* fstatus, DecBlock* blocks, DecUnit* units, uint32_t* fwant,
                              const uint64_t* ftok, hipStream_t st) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_dframe_fill, dim3(cdiv(n, 256)), dim3(256), 0, st, src, frame_off, frame_len, n, dst_off,
                       dst_cap, blk_base, fstatus, blocks, units, fwant, ftok);
    return hipGetLastError();
}
hipError_t launch_dframe_finish(const uint64_t* blk_base, uint32_t n, const uint32_t* nblk, const DecBlock* blocks,
                                const uint32_t* blk_out, const int32_t* blk_status, int32_t* fstatus,
                                uint32_t* out_len, hipStream_t st) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_dframe_finish, dim3(cdiv(n, 256)), dim3(256), 0, st, blk_base, n, nblk, blocks, blk_out,
                       blk_status, fstatus, out_len);
    return hipGetLastError();
}
hipError_t launch_dframe_close(const uint8_t* src, const uint64_t* frame_off, const uint64_t* blk_base,
                               const uint32_t* nblk, const DecBlock* blocks, const uint32_t* blk_out,
                               const int32_t* blk_status, const uint64_t* blk_hash, const uint8_t* out,
                               const uint64_t* out_off, const uint32_t* fwant, uint32_t n, const int32_t* fstat_in,
                               int32_t* fstatus, uint32_t* out_len, uint32_t* got_hash, hipStream_t st,
                               uint32_t* pend) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_dframe_close, dim3(cdiv((uint64_t)n * kCloseLanes, 64)), dim3(64), 0, st, src, frame_off, blk_base, nblk,
                       blocks, blk_out, blk_status, blk_hash, out, out_off, fwant, n, fstat_in, fstatus, out_len,
                       got_hash, pend);
    return hipGetLastError();
}
hipError_t launch_dframe_verify(const uint8_t* src, const uint64_t* frame_off, uint32_t n, const uint32_t* fwant,
                                const uint32_t* got, const uint32_t* out_len, int32_t* fstatus, hipStream_t st) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_dframe_verify, dim3(cdiv(n, 256)), dim3(256), 0, st, src, frame_off, n, fwant, got, out_len,
                       fstatus);
    return hipGetLastError();
}
}  // namespace s3hc

#ifdef S3HC_PROF
extern "C" int s3hc_diag_prof(unsigned long long* out, int n, int reset) {
    if (n > 32) n = 32;
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(s3hc::g_prof), sizeof(unsigned long long) * n) != hipSuccess) return -1;
    if (reset) {
        unsigned long long z[32] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(s3hc::g_prof), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#endif

// The 64 KiB-block fast path and the small-batch decoder (same translation unit: k_djump runs
// decode_unit_pe for the blocks its token index does not take).
#include "s3hc_fast.hip"
