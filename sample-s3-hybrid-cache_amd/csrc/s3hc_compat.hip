// lz4_flex-compatible frame encoder ("compat" encoder).
//
// Emits the frames lz4_flex 0.11 FrameEncoder writes for compress_with_algorithm
// (compression.rs:530-591: FrameInfo{content_checksum, Independent}, BlockSize::Auto from the
// whole-buffer write) with block payloads byte-identical to lz4_flex's greedy block compressor
// (block/compress.rs compress_internal, HashTable4K, hash5, skip acceleration, backtracking),
// as restated in oracle/lz4_oracle.c:173-279 (or_lz4flex_compress_frame). The restatement is
// recalled, not verified against lz4_flex source, so compressed-byte parity
// with the real crate stays "unpinned"; parity with the oracle is tested bit-exact.
//
// The algorithm is serial by definition (each hash-table read depends on the writes of every
// earlier attempt), so the unit is one frame per wave and the wave speculates over the serial
// loop instead of parallelising the block:
//   * scan: the 64 lanes take the next 64 attempt positions of the skip schedule (attempt i of a
//     scan is at cur + i + 16q(q-1) + q*r, q = i/32, r = i%32: step = 1 + i/32), hash them and
//     read the LDS table; a lane whose hash an earlier lane of the batch also hashed takes that
//     lane's position as its candidate (what the serial writes would have left); the first lane
//     whose candidate verifies is the serial loop's match; the table writes of the lanes up to it
//     are committed (the last of equal hashes wins). In-batch hash collisions are detected with
//     a tag write/read-back and resolved by a 63-step shuffle only when present.
//   * backtrack, forward match length, literal and length-byte copies: 64 bytes per wave step.
// Entries written by earlier blocks of the frame are always rejected (stale or out of range),
// so a block whose output would not be smaller than its input stops early and is stored.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace s3hc {
namespace compat {

constexpr uint32_t kTbl = 4096;     // HashTable4K
constexpr uint32_t kTagShift = 1;   // duplicate-detection tags: one per 2 table slots (false flags only cost the resolution pass)
constexpr uint32_t kMinMatch = 4;   // MINMATCH
constexpr uint32_t kMfLimit = 12;   // MFLIMIT
constexpr uint32_t kEndOffset = 6;  // LAST_LITERALS + 1
constexpr uint32_t kMaxDist = 65535;
#ifndef S3HC_COMPAT_BATCH
#define S3HC_COMPAT_BATCH 32
#endif
constexpr uint32_t kBatch = S3HC_COMPAT_BATCH;  // attempts speculated per wave step (<= 64)

__device__ __forceinline__ int lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0)); }
__device__ __forceinline__ uint32_t rdl(uint32_t v, uint32_t l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l);
}
__device__ __forceinline__ uint32_t shfl(uint32_t v, int src) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute(src << 2, (int)v);
}
// Unaligned reads from two aligned dwords (the dword holding p and the next one: never past
// p + 7, which every caller keeps inside its block).
struct W5 {
    uint32_t lo, b4;  // bytes p..p+3 (LE), byte p+4
};
__device__ __forceinline__ W5 ld5(const uint8_t* p) {
    const uintptr_t a = (uintptr_t)p;
    const uint32_t* w = (const uint32_t*)(a & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(a & 3), w0 = w[0], w1 = w[1];
    return W5{__builtin_amdgcn_alignbyte(w1, w0, sh), (w1 >> (8 * sh)) & 0xFFu};
}
__device__ __forceinline__ uint32_t ld32(const uint8_t* p) { return ld5(p).lo; }
// hash5 >> HASHTABLE_BIT_SHIFT_4K over the 5 low bytes of the u64 at p (oracle hash5_idx)
// In 32-bit halves: X = seq << 24 (X_lo = lo << 24, X_hi = lo >> 8 | b4 << 24), P = 207·2^32 +
// 465362107. The table index is hash5 >> 4 = bits 52..63 of X·P (the oracle's >> 48 then >> 4),
// i.e. bits 20..31 of the high word hi = X_hi·P_lo + X_lo·207 + mulhi(X_lo, P_lo) (mod 2^32).
__device__ __forceinline__ uint32_t hash5w(W5 v) {
    const uint32_t xl = v.lo << 24, xh = (v.lo >> 8) | (v.b4 << 24);
    const uint32_t hi = xh * 465362107u + xl * 207u + __umulhi(xl, 465362107u);
    return hi >> 20;
}
__device__ __forceinline__ uint32_t hash5(const uint8_t* p) { return hash5w(ld5(p)); }

// Output sink of one block: `sp` bytes written, `cap` = largest payload still worth keeping
// (one less than the block), uniform across the wave. false = overflow (the block is stored).
struct Sink {
    uint8_t* out;
    uint32_t sp, cap;
    __device__ __forceinline__ bool byte(uint32_t b, int lane) {
        if (sp >= cap) return false;
        if (lane == 0) out[sp] = (uint8_t)b;
        ++sp;
        return true;
    }
    __device__ __forceinline__ bool copy(const uint8_t* src, uint32_t n, int lane) {
        if (cap - sp < n) return false;
        for (uint32_t t = (uint32_t)lane; t < n; t += 64) out[sp + t] = src[t];
        sp += n;
        return true;
    }
    // write_integer: n / 255 bytes of 0xFF, then n % 255
    __device__ __forceinline__ bool integer(uint32_t n, int lane) {
        const uint32_t k = n / 255u;
        if (cap - sp < k + 1) return false;
        for (uint32_t t = (uint32_t)lane; t < k; t += 64) out[sp + t] = 0xFF;
        if (lane == 0) out[sp + k] = (uint8_t)(n - 255u * k);
        sp += k + 1;
        return true;
    }
    __device__ __forceinline__ bool last_literals(const uint8_t* in, uint32_t len, uint32_t start, int lane) {
        const uint32_t lit = len - start;
        if (!byte(lit < 15u ? lit << 4 : 0xF0u, lane)) return false;
        if (lit >= 15u && !integer(lit - 15u, lane)) return false;
        return copy(in + start, lit, lane);
    }
};

// lzf_compress_internal (oracle/lz4_oracle.c:173-231) for one block; returns false when the
// payload would not be smaller than the block (or the table rejects nothing but it overflows).
template <typename TE>
__device__ bool compress_block(const uint8_t* __restrict__ in, uint32_t len, uint32_t so, TE* dict,
                               uint8_t* tag, Sink& s, int lane) {
    if (len < kMfLimit + 1) return s.last_literals(in, len, 0, lane);
    const uint32_t end_pos_check = len - kMfLimit;
    uint32_t lit_start = 0, cur = 0;
    if (so == 0) {  // "we can't start with a match": position 0 inserted, scanning starts at 1
        if (lane == 0) dict[hash5(in)] = 0;
        cur = 1;
    }
    __builtin_amdgcn_wave_barrier();
    for (;;) {
        // ---- scan (speculative over 64 attempts of the skip schedule)
        uint32_t mpos = 0, mcand = 0;
        for (uint32_t i0 = 0;; i0 += kBatch) {
            const uint32_t i = i0 + (uint32_t)lane, q = i >> 5, r = i & 31u;
            const uint32_t p = cur + i + 16u * q * (q ? q - 1u : 0u) + q * r;
            const bool valid = (uint32_t)lane < kBatch && p <= end_pos_check;
            const W5 wp = valid ? ld5(in + p) : W5{0u, 0u};
            const uint32_t h = hash5w(wp);
            // volatile: the read-back must see other lanes' tag writes, not this lane's own
            volatile TE* vd = dict;
            volatile uint8_t* vt = tag;
            const uint32_t old = valid ? (uint32_t)vd[h] : 0u;
            if (valid) vt[h >> kTagShift] = (uint8_t)lane;
            __builtin_amdgcn_wave_barrier();
            const uint64_t cm = __ballot(valid && vt[h >> kTagShift] != (uint8_t)lane);
            // Every lane whose candidate an earlier in-batch duplicate changes sits at or after the
            // first flagged lane `lo`: a match found before `lo` with the table's candidates is the
            // serial loop's, and no two lanes up to it share a hash.
            const uint32_t lo = cm ? (uint32_t)__builtin_ctzll(cm) : 64u;
            uint32_t cand = old;
            bool m = valid && (so + p - cand <= kMaxDist) && (cand >= so) && ld32(in + (cand - so)) == wp.lo;
            uint64_t mb = __ballot(m);
            uint32_t k = mb ? (uint32_t)__builtin_ctzll(mb) : 64u;
            if (cm && k >= lo) {
                // previous lane of the batch with the same hash (invalid lanes carry a sentinel
                // that matches nothing)
                const uint32_t hv = valid ? h : 0x10000u | (uint32_t)lane;
                int prev_dup = -1;
                for (int d = 1; d < (int)kBatch; ++d) {
                    const uint32_t hp = shfl(hv, lane - d);
                    if (prev_dup < 0 && lane - d >= 0 && hp == hv) prev_dup = lane - d;
                }
                const uint32_t pp = shfl(p, prev_dup < 0 ? lane : prev_dup);
                if (valid && prev_dup >= 0) {
                    cand = pp + so;
                    m = (so + p - cand <= kMaxDist) && (cand >= so) && ld32(in + (cand - so)) == wp.lo;
                }
                mb = __ballot(m);
                k = mb ? (uint32_t)__builtin_ctzll(mb) : 64u;
            }
            const uint32_t cb = cand - so;
            // commit the table writes of attempts <= k. Equal hashes: every committing lane
            // stores, then lanes still seeing a smaller position of their group store again, so
            // the slot ends with the group's last (largest) position, as the serial writes leave it
            const bool commit = valid && (uint32_t)lane <= k;
            if (commit) vd[h] = (TE)(p + so);
            if (cm) {
                for (;;) {
                    __builtin_amdgcn_wave_barrier();
                    const bool fix = commit && (uint32_t)vd[h] < p + so;
                    if (!__ballot(fix)) break;
                    if (fix) vd[h] = (TE)(p + so);
                }
            }
            __builtin_amdgcn_wave_barrier();
            if (mb) {
                mpos = rdl(p, k);
                mcand = rdl(cb, k);
                break;
            }
            if (__ballot(!valid && (uint32_t)lane < kBatch))  // cur > end_pos_check
                return s.last_literals(in, len, lit_start, lane);
        }
        // ---- backtrack_match and count_same_bytes, both probed in the same round trip.
        // The count starts at the backtracked position + 4; its first b bytes lie in the
        // backtracked + verified run, so dup = b + F with F the equal run from mpos + 4.
        uint32_t c = mpos, cd = mcand;
        const uint32_t blim = cd < c - lit_start ? cd : c - lit_start;
        const uint32_t flim = len - kEndOffset > c + kMinMatch ? len - kEndOffset - (c + kMinMatch) : 0u;
        uint32_t b, F;
        {
            const uint32_t t = (uint32_t)lane;
            const bool bne = t < blim && in[c - 1 - t] != in[cd - 1 - t];
            const bool fne = t < flim && in[c + kMinMatch + t] != in[cd + kMinMatch + t];
            const uint64_t nb = __ballot(bne), nf = __ballot(fne);
            b = nb ? (uint32_t)__builtin_ctzll(nb) : 64u;
            F = nf ? (uint32_t)__builtin_ctzll(nf) : 64u;
        }
        if (b == 64u) {  // backtrack run of 64+ bytes
            while (b < blim) {
                const uint32_t t = b + (uint32_t)lane;
                const uint64_t neq = __ballot(t < blim && in[c - 1 - t] != in[cd - 1 - t]);
                if (neq) { b += (uint32_t)__builtin_ctzll(neq); break; }
                b += 64;
            }
        }
        b = b < blim ? b : blim;
        if (F == 64u) {  // match of 68+ bytes
            while (F < flim) {
                const uint32_t t = F + (uint32_t)lane;
                const uint64_t neq = __ballot(t < flim && in[c + kMinMatch + t] != in[cd + kMinMatch + t]);
                if (neq) { F += (uint32_t)__builtin_ctzll(neq); break; }
                F += 64;
            }
        }
        F = F < flim ? F : flim;
        c -= b;
        cd -= b;
        const uint32_t lit_len = c - lit_start;
        const uint32_t offset = c - cd;
        const uint32_t dup = b + F;
        c += kMinMatch + dup;
        if (lane == 0) ((volatile TE*)dict)[hash5(in + c - 2)] = (TE)(c - 2 + so);
        __builtin_amdgcn_wave_barrier();
        // ---- sequence
        const uint32_t token = ((lit_len < 15u ? lit_len : 15u) << 4) | (dup < 15u ? dup : 15u);
        if (!s.byte(token, lane)) return false;
        if (lit_len >= 15u && !s.integer(lit_len - 15u, lane)) return false;
        if (!s.copy(in + lit_start, lit_len, lane)) return false;
        if (!s.byte(offset & 0xFFu, lane) || !s.byte(offset >> 8, lane)) return false;
        if (dup >= 15u && !s.integer(dup - 15u, lane)) return false;
        lit_start = c;
        cur = c;
    }
}

// One wave per frame: FrameEncoder(FrameInfo{content_checksum, Independent}) + write_all +
// finish (oracle/lz4_oracle.c:242-279). fhash[f] = xxh32 of the frame's input (seed 0).
// TE = table entry: u16 for frames of <= 64 KiB (positions < 2^16; 12 KiB of LDS per wave,
// 13 waves/CU), u32 otherwise (positions + stream offset; 20 KiB, 8 waves/CU). A launch
// encodes the frames of its class and skips the others.
template <typename TE>
__global__ __launch_bounds__(64) void k_compat_frames(const uint8_t* __restrict__ src, const uint64_t* __restrict__ src_off,
                                                      const uint32_t* __restrict__ len, uint32_t n, uint8_t* __restrict__ dst,
                                                      const uint64_t* __restrict__ dst_off,
                                                      const uint32_t* __restrict__ fhash, uint32_t* __restrict__ frame_len) {
    __shared__ TE dict[kTbl];
    __shared__ uint8_t tag[kTbl >> kTagShift];
    const uint32_t f = blockIdx.x;
    if (f >= n) return;
    const uint32_t N = len[f];
    if ((N <= 65536u) != (sizeof(TE) == 2)) return;
    const int lane = lane_id();
    const uint8_t* in0 = src + src_off[f];
    uint8_t* o = dst + dst_off[f];
    for (uint32_t t = (uint32_t)lane; t < kTbl; t += 64) dict[t] = 0;  // calloc'd table
    // BlockSize::from_buf_length: <= 64 KiB -> Max64KB, <= 256 KiB -> Max256KB, else Max4MB
    const uint32_t code = N <= 65536u ? 4u : (N <= 262144u ? 5u : 7u);
    const uint32_t bmax = 1u << (16 + 2 * (code - 4));
    if (lane < 7) {
        // magic 04 22 4D 18, FLG 0x64, BD, HC = (xxh32([FLG, BD]) >> 8) as u8
        const uint8_t hc = code == 4 ? 0xA7 : (code == 5 ? 0x08 : 0xB9);
        const uint8_t hdr[7] = {0x04, 0x22, 0x4D, 0x18, 0x64, (uint8_t)(code << 4), hc};
        o[lane] = hdr[lane];
    }
    __syncthreads();
    uint64_t op = 7;
    for (uint32_t so = 0; so < N; so += bmax) {
        const uint32_t blen = N - so < bmax ? N - so : bmax;
        const uint8_t* in = in0 + so;
        Sink s{o + op + 4, 0, blen - 1};
        const bool ok = compress_block(in, blen, so, dict, tag, s, lane);
        uint32_t word, body;
        if (ok) {
            word = s.sp;
            body = s.sp;
        } else {  // stored: comp_len >= src.len()
            __threadfence_block();
            for (uint32_t t = (uint32_t)lane; t < blen; t += 64) o[op + 4 + t] = in[t];
            word = blen | 0x80000000u;
            body = blen;
        }
        if (lane < 4) o[op + lane] = (uint8_t)(word >> (8 * lane));
        op += 4 + body;
    }
    const uint32_t xh = fhash[f];
    if (lane < 8) o[op + lane] = lane < 4 ? 0 : (uint8_t)(xh >> (8 * (lane - 4)));  // EndMark, checksum
    if (lane == 0) frame_len[f] = (uint32_t)(op + 8);
}

}  // namespace compat

hipError_t launch_compat_frames(const uint8_t* src, const uint64_t* src_off, const uint32_t* len, uint32_t n,
                                uint8_t* dst, const uint64_t* dst_off, const uint32_t* fhash, uint32_t* frame_len,
                                uint32_t n_small, hipStream_t st) {
    if (!n) return hipSuccess;
    if (n_small)
        hipLaunchKernelGGL(compat::k_compat_frames<uint16_t>, dim3(n), dim3(64), 0, st, src, src_off, len, n, dst,
                           dst_off, fhash, frame_len);
    if (n_small < n)
        hipLaunchKernelGGL(compat::k_compat_frames<uint32_t>, dim3(n), dim3(64), 0, st, src, src_off, len, n, dst,
                           dst_off, fhash, frame_len);
    return hipGetLastError();
}

}  // namespace s3hc
